// pss_pipeline.hip -- fused filterbank synthesis engine for MI355X (gfx950).
//
// One PssPipeline run = source -> [FFT delay ramp] -> [null] -> [noise] -> data.
// See include/pss_hip.h for the ABI and DESIGN.md for the kernel/roofline
// discussion.  Paths:
//   * no delay stage           : k_elementwise          (1 HBM pass)
//   * N = 2^m, 64 <= N <= 8192 : k_single<L>            (1 HBM pass, FFT in LDS)
//   * N = 2^m, N >= 16384      : k_colA -> k_row -> k_colC  (four-step, 2 spills)
//   * 2^m x {6..60} (smooth)   : mixed-radix four-step
//   * other even N <= 8192     : direct DFT              (O(N^2) in LDS tiles)
//   * other even N >  8192     : Bluestein chirp-z through a 2^m four-step
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <math.h>
#include <type_traits>


#include "pss_engine.hpp"

using namespace pss;

// ---------------------------------------------------------------------------
// error reporting
// ---------------------------------------------------------------------------
static thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}


// ---------------------------------------------------------------------------
// opt-in per-kernel timing (bench.py): hipEvents recorded on the launch stream
// around every kernel of pss_run, summed per kernel kind on collect.
// ---------------------------------------------------------------------------
static bool g_timing = false;
struct TimedLaunch { int kind; int64_t units; hipEvent_t a, b; };
static TimedLaunch g_tl[4096];
static int g_ntl = 0;
static int g_tk_pending = -1;

static int64_t g_tk_units = 0;   // samples processed by the launch being timed

// (the events are created once per slot and reused: creating two events per
// launch inside the timed steps cost the host ~tens of microseconds each)
void tk_begin(int kind, hipStream_t st) {
    if (!g_timing || g_ntl >= 4096) { g_tk_pending = -1; return; }
    TimedLaunch &t = g_tl[g_ntl];
    if (!t.a && hipEventCreate(&t.a) != hipSuccess) { t.a = nullptr; g_tk_pending = -1; return; }
    if (!t.b && hipEventCreate(&t.b) != hipSuccess) { t.b = nullptr; g_tk_pending = -1; return; }
    t.kind = kind;
    t.units = g_tk_units;
    (void)hipEventRecord(t.a, st);
    g_tk_pending = kind;
}
void tk_end(hipStream_t st) {
    if (g_tk_pending < 0) return;
    (void)hipEventRecord(g_tl[g_ntl].b, st);
    ++g_ntl;
    g_tk_pending = -1;
}

int g_flags = 0;   // pss_set_flags (test hook)

// launch-plan log: one line per pss_run since the last pss_plan_collect
static char g_plan[16384];
static size_t g_plan_len = 0;
void plan_note(const char *fmt, ...) {
    if (g_plan_len + 1 >= sizeof(g_plan)) return;
    va_list ap;
    va_start(ap, fmt);
    const int w = vsnprintf(g_plan + g_plan_len, sizeof(g_plan) - g_plan_len, fmt, ap);
    va_end(ap);
    if (w > 0) g_plan_len = std::min(g_plan_len + (size_t)w, sizeof(g_plan) - 1);
}

SideStreams *side_streams() {
    static SideStreams g[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    SideStreams &x = g[dev];
    if (!x.ok) {
        for (int i = 0; i < 2; ++i)
            if (hipStreamCreateWithFlags(&x.s[i], hipStreamNonBlocking) != hipSuccess) return nullptr;
        for (int i = 0; i < 40; ++i)
            if (hipEventCreateWithFlags(&x.ev[i], hipEventDisableTiming) != hipSuccess) return nullptr;
        x.ok = true;
    }
    return &x;
}

// Delayed null: the (pre-shift) box mask is the same for every channel, so it
// is evaluated once per run into a row of N floats (0 outside the boxes) that
// the source stage of every channel reads.
__global__ __launch_bounds__(256) void k_box_row(KP k, float *row) {
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < k.N;
         n += (int64_t)gridDim.x * blockDim.x) {
        int rk, j;
        row[n] = box_of(k, n, rk, j) ? box_value(k, n, rk, j) : 0.0f;
    }
}

int launch_box_row(const KP &k, float *row, hipStream_t st) {
    k_box_row<<<stream_grid(k.N, 1), dim3(256), 0, st>>>(k, row);
    LAUNCHCHK();
    return PSS_OK;
}

// ---------------------------------------------------------------------------
// path 0: no FFT -- source -> null(undelayed) -> epilogue, one pass
// ---------------------------------------------------------------------------
// With k.mtab (delayed null on a four-step length whose data needs no delay
// in this run) the mask decisions come from the mask table.
__global__ __launch_bounds__(256) void k_elementwise(KP k) {
    const int r = blockIdx.y;
    const int64_t items = (k.N + 3) >> 2;
    uint32_t is = 0;
    float t = 0.f;
    if (k.mtab) mask_split((uint64_t)k.p.mask_ramp[r], k.log2n, is, t);
    for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < items;
         it += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n0 = it << 2;
        const int cnt = (int)min((int64_t)4, k.N - n0);
        float re[4], im[4];
        source4(k, r, n0, cnt, re, im, true, !k.mtab);
        if (k.mtab) {
            const uint32_t h = mask_hits4(k, n0, is, t);
#pragma unroll
            for (int i = 0; i < 4; ++i) im[i] = ((h >> i) & 1u) ? 2.0f : 0.0f;
        }
        epilogue4(k, r, n0, cnt, re, im, false);
    }
}

int launch_elementwise(const KP &k, hipStream_t st) {
    dim3 g = stream_grid((k.N + 3) / 4, k.p.nchan);
    plan_note(k.mtab ? " elementwise" : "elementwise");
    tk_begin(TK_ELEM, st);
    k_elementwise<<<g, dim3(256), 0, st>>>(k);
    tk_end(st);
    LAUNCHCHK();
    return PSS_OK;
}

// ---------------------------------------------------------------------------
// utility kernels
// ---------------------------------------------------------------------------
__global__ void k_down_sample(const float *in, float *out, int64_t in_len, int64_t in_ld,
                              int32_t fact) {
    const int r = blockIdx.y;
    const int64_t nout = in_len / fact;
    const float *row = in + (int64_t)r * in_ld;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nout;
         i += (int64_t)gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int j = 0; j < fact; ++j) s += row[i * fact + j];
        out[(int64_t)r * nout + i] = (float)(s / fact);
    }
}

__global__ void k_rebin(const float *in, float *out, int64_t in_ld, int32_t newlen,
                        const int64_t *lo, const int64_t *hi) {
    const int r = blockIdx.y;
    const float *row = in + (int64_t)r * in_ld;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < newlen; i += gridDim.x * blockDim.x) {
        double s = 0.0;
        const int64_t a = lo[i], b = hi[i];
        PSS_DASSERT(a >= 0 && a <= b && b <= in_ld);
        for (int64_t j = a; j < b; ++j) s += row[j];
        out[(int64_t)r * newlen + i] = (b > a) ? (float)(s / (double)(b - a)) : NAN;
    }
}

// observe()'s resampled copy, last step of a run with out_len > 0: bin i of
// row r = (window sum) / (window width), clipped from above at `clip` in
// float64 (the reference clips its float64 `out`), cast to float32 or int8
// (k_clip_cast's int8 rule); an empty window gives NaN (np.nanmean).
__global__ void k_out_finalize(const double *acc, const int64_t *lo, const int64_t *hi, double step, void *out,
                               int64_t len, int64_t total, float clip, int32_t kind) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e % len;
        const double w = lo ? (double)(hi[i] - lo[i]) : step;
        double v = w > 0.0 ? acc[e] / w : __builtin_nan("");
        if (v > (double)clip) v = (double)clip;
        if (kind == PSS_OUT_F32) {
            ((float *)out)[e] = (float)v;
        } else {
            // clamp and truncate the float64 mean itself, as the reference's
            // np.array(out, dtype=int8) casts its float64 out (a float32
            // rounding first could carry a mean just below an integer up to it)
            ((int8_t *)out)[e] = (int8_t)(int)trunc(fmin(fmax(v, -128.0), 127.0));
        }
    }
}

__global__ void k_clip_cast(const float *in, void *out, int64_t count, float clip, int32_t kind) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (int64_t)gridDim.x * blockDim.x) {
        float v = in[i];
        v = (v > clip) ? clip : v;
        if (kind == PSS_OUT_F32) {
            ((float *)out)[i] = v;
        } else {
            v = fminf(fmaxf(v, -128.f), 127.f);
            ((int8_t *)out)[i] = (int8_t)(int)truncf(v);
        }
    }
}

__global__ void k_fold(const float *data, float *out, int64_t ld, int64_t npbins, int64_t n_fold) {
    const int c = blockIdx.y;
    const int64_t half = npbins / 2;
    const float *row = data + (int64_t)c * ld + npbins;
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < half;
         b += (int64_t)gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int64_t f = 0; f < n_fold; ++f) s += row[f * half + b];
        out[(int64_t)c * half + b] = (float)s;
    }
}

// Whole-period fold: out[c][b] = sum_{p < nper} data[c][p nbin + b], float64
// accumulation in 8 independent partial sums (8 loads in flight per lane;
// adjacent lanes read adjacent bins).
__global__ void k_fold_periods(const float *data, float *out, int64_t ld, int64_t nbin, int64_t nper) {
    const int c = blockIdx.y;
    const float *row = data + (int64_t)c * ld;
    for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nbin;
         b += (int64_t)gridDim.x * blockDim.x) {
        double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int64_t p = 0;
        for (; p + 8 <= nper; p += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) s[u] += row[(p + u) * nbin + b];
        }
        for (; p < nper; ++p) s[0] += row[p * nbin + b];
        out[(int64_t)c * nbin + b] = (float)(((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7])));
    }
}

// shift_val = count/2 - argmax(row[0:count]) with the reference's failure
// cases flagged (non-unique maximum, NaN); one workgroup
__global__ __launch_bounds__(256) void k_null_shift(const float *row, int64_t count, int64_t *out) {
    __shared__ float smax[256];
    __shared__ int sidx[256], scnt[256], snan[256];
    float m = -INFINITY;
    int idx = -1, cnt = 0, nan = 0;
    for (int64_t i = threadIdx.x; i < count; i += 256) {
        const float v = row[i];
        if (v != v) { nan = 1; continue; }
        if (v > m) { m = v; idx = (int)i; cnt = 1; }
        else if (v == m) { ++cnt; }
    }
    smax[threadIdx.x] = m;
    sidx[threadIdx.x] = idx;
    scnt[threadIdx.x] = cnt;
    snan[threadIdx.x] = nan;
    __syncthreads();
    if (threadIdx.x == 0) {
        float M = -INFINITY;
        int I = -1, C = 0, Nn = 0;
        for (int t = 0; t < 256; ++t) {
            Nn |= snan[t];
            if (scnt[t] == 0) continue;
            if (smax[t] > M) { M = smax[t]; I = sidx[t]; C = scnt[t]; }
            else if (smax[t] == M) { C += scnt[t]; if (sidx[t] < I) I = sidx[t]; }
        }
        out[0] = count / 2 - (int64_t)(I < 0 ? 0 : I);
        out[1] = Nn ? 2 : (C != 1 ? 1 : 0);
    }
}

__global__ void k_chi2_fill(float *out, int64_t n, int32_t chan0, float df, uint64_t seed,
                            uint32_t call_id, uint32_t purpose) {
    const int r = blockIdx.y;
    Rng g(seed, call_id, purpose);
    const int64_t items = (n + 3) >> 2;
    for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < items;
         it += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n0 = it << 2;
        float x[4];
        draw4(g, n0, (uint32_t)(chan0 + r), df, x);
        for (int i = 0; i < 4 && n0 + i < n; ++i) out[(int64_t)r * n + n0 + i] = x[i];
    }
}

extern "C" int64_t pss_workspace_bytes(int32_t nchan, int64_t nsamp);

static int validate(const PssPipeline *p) {
    if (!p) return fail(PSS_EINVAL, "null pipeline");
    if (p->nchan <= 0 || p->nsamp <= 0) return fail(PSS_EINVAL, "empty signal (%d x %lld)", p->nchan, (long long)p->nsamp);
    if (p->nchan > 65535) return fail(PSS_EINVAL, "nchan %d > 65535 per launch", p->nchan);
    if (!p->data) return fail(PSS_EINVAL, "data is NULL");
    if (p->ld < p->nsamp) return fail(PSS_EINVAL, "ld < nsamp");
    if (p->nsamp >= (1ll << 31)) return fail(PSS_EUNSUPPORTED, "nsamp >= 2^31");
    if (p->src == PSS_SRC_SEARCH && (!p->prof || p->nint < 1 || p->knot_m < 1))
        return fail(PSS_EINVAL, "search source needs a PCHIP table");
    if (p->src == PSS_SRC_FOLD && (!p->prof || p->nph < 1))
        return fail(PSS_EINVAL, "fold source needs a profile table");
    if (p->prof_split && (p->src != PSS_SRC_SEARCH || p->gen_amp == 2 || p->knot_m != (uint32_t)p->nint))
        return fail(PSS_EINVAL, "split-cell profile tables are for the PCHIP search source with knot_m == nint");
    if ((p->src == PSS_SRC_SEARCH || p->src == PSS_SRC_FOLD) && p->gen_amp != 2 && p->prof_rows != 1 &&
        (p->prof_rows < 1 || p->prof_row0 < 0 || p->prof_row0 > p->chan0 ||
         (int64_t)p->chan0 + p->nchan - p->prof_row0 > (int64_t)p->prof_rows))
        return fail(PSS_EINVAL, "profile table rows [%d, %d) do not cover channels [%d, %d)", p->prof_row0,
                    p->prof_row0 + p->prof_rows, p->chan0, p->chan0 + p->nchan);
    if (p->null_mode != PSS_NULL_NONE && (!p->null_rank || p->nph < 1))
        return fail(PSS_EINVAL, "null needs null_rank and nph");
    if (p->null_mode == PSS_NULL_DELAYED && !p->shift)
        return fail(PSS_EINVAL, "delayed null needs the FFT delay stage");
    if (p->shift) {
        if (p->nsamp & 1)
            return fail(PSS_EINVAL, "odd N=%lld: the reference's irfft returns N-1 samples", (long long)p->nsamp);
        if (!p->htab && (!p->ramp || !p->nyq_re || !p->nyq_im))
            return fail(PSS_EINVAL, "shift needs ramp/nyq arrays");
        if (p->htab && (p->nsamp > (1ll << 24) || p->null_mode != PSS_NULL_NONE))
            return fail(PSS_EUNSUPPORTED, "transfer-function run: N=%lld, null %d", (long long)p->nsamp,
                        p->null_mode);
        if (!p->work) return fail(PSS_EINVAL, "shift needs a workspace");
        if (p->nsamp > (1ll << 24) && !is_pow2(p->nsamp))
            return fail(PSS_EUNSUPPORTED, "N=%lld", (long long)p->nsamp);
        if (p->null_mode == PSS_NULL_DELAYED && fourstep_len(p->nsamp) && !p->mask_ramp)
            return fail(PSS_EINVAL, "delayed null needs mask_ramp");
        if (p->tail_a && p->null_mode == PSS_NULL_DELAYED && !fourstep_len(p->nsamp))
            return fail(PSS_EUNSUPPORTED, "scattering tail with a delayed null at N=%lld (the mask shares the "
                        "filtered transform off the four-step lengths)", (long long)p->nsamp);
    }
    if (p->out_kind != PSS_OUT_NONE && !p->out) return fail(PSS_EINVAL, "out is NULL");
    if (p->out_kind != PSS_OUT_NONE && p->out_len > 0) {
        if (!p->out_acc) return fail(PSS_EINVAL, "resampled out needs out_acc");
        if ((p->out_lo == nullptr) != (p->out_hi == nullptr)) return fail(PSS_EINVAL, "out_lo / out_hi");
        if (!(p->out_step >= 1.0)) return fail(PSS_EINVAL, "out_step %g < 1", p->out_step);
        if (!p->out_lo && (p->out_step != floor(p->out_step) || p->out_step * p->out_len > (double)p->nsamp))
            return fail(PSS_EINVAL, "uniform windows: integer out_step with out_len * out_step <= nsamp");
    }
    return PSS_OK;
}

extern "C" {

int pss_version(void) { return 100; }

// sha256 of the library's sources (psrsigsim_amd/build.py), so a loader can
// tell whether this binary was built from the sources next to it
#ifndef PSS_BUILD_HASH
#define PSS_BUILD_HASH "unknown"
#endif
const char *pss_build_hash(void) { return "PSS_BUILD_HASH=" PSS_BUILD_HASH; }

int pss_set_flags(int flags) {
    const int old = g_flags;
    g_flags = flags;
    return old;
}

void pss_timing_enable(int on) {
    g_timing = on != 0;
    // create the first slots' events now, not inside the first timed run
    for (int i = 0; g_timing && i < 512; ++i) {
        if (!g_tl[i].a && hipEventCreate(&g_tl[i].a) != hipSuccess) g_tl[i].a = nullptr;
        if (!g_tl[i].b && hipEventCreate(&g_tl[i].b) != hipSuccess) g_tl[i].b = nullptr;
    }
}

double pss_timing_span_ms(void) {
    if (g_ntl < 1) return 0.0;
    float e = 0.f;
    (void)hipEventSynchronize(g_tl[g_ntl - 1].b);
    if (hipEventElapsedTime(&e, g_tl[0].a, g_tl[g_ntl - 1].b) != hipSuccess) return -1.0;
    return e;
}

int pss_timing_collect(int32_t *kind, double *ms, int64_t *units, int cap) {
    int n = 0;
    for (int i = 0; i < g_ntl; ++i) {
        TimedLaunch &t = g_tl[i];
        float e = 0.f;
        (void)hipEventSynchronize(t.b);
        (void)hipEventElapsedTime(&e, t.a, t.b);
        if (n < cap) { kind[n] = t.kind; ms[n] = e; units[n] = t.units; ++n; }
    }
    g_ntl = 0;
    return n;
}

int pss_plan_collect(char *buf, size_t n) {
    const int len = (int)g_plan_len;
    if (buf && n) {
        const size_t c = std::min(n - 1, g_plan_len);
        memcpy(buf, g_plan, c);
        buf[c] = 0;
    }
    g_plan_len = 0;
    g_plan[0] = 0;
    return len;
}

int pss_last_error(char *buf, size_t n) {
    if (buf && n) {
        strncpy(buf, g_err, n - 1);
        buf[n - 1] = 0;
    }
    return (int)strlen(g_err);
}

int64_t pss_workspace_bytes(int32_t nchan, int64_t nsamp) {
    if (nchan <= 0 || nsamp <= 0) return 0;
    return ws_layout(nchan, nsamp).total;
}

static int run_paths(const PssPipeline *p, hipStream_t st);

int pss_run(const PssPipeline *p, void *stream) {
    int rc = validate(p);
    if (rc) return rc;
    if (g_plan_len) plan_note("\n");
    plan_note("%dx%lld: ", p->nchan, (long long)p->nsamp);
    hipStream_t st = (hipStream_t)stream;
    const bool windows = p->out_kind != PSS_OUT_NONE && p->out_len > 0;
    if (windows) HIPCHK(hipMemsetAsync(p->out_acc, 0, (size_t)p->nchan * (size_t)p->out_len * 8, st));
    rc = run_paths(p, st);
    if (rc || !windows) return rc;
    const int64_t total = (int64_t)p->nchan * p->out_len;
    k_out_finalize<<<stream_grid(total, 1), dim3(256), 0, st>>>(p->out_acc, p->out_lo, p->out_hi, p->out_step,
                                                                 p->out, p->out_len, total, p->clip, p->out_kind);
    LAUNCHCHK();
    return PSS_OK;
}

static int run_paths(const PssPipeline *p, hipStream_t st) {
    KP k;
    memset(&k, 0, sizeof(k));
    k.p = *p;
    k.N = p->nsamp;
    k.N1 = 1;
    k.N2 = p->nsamp;
    k.invN = (float)(1.0 / (double)p->nsamp);
    g_tk_units = (int64_t)p->nchan * p->nsamp;
    if (!p->shift) {
        return launch_elementwise(k, st);
    }
    const int64_t N = p->nsamp;
    float *row = reinterpret_cast<float *>(reinterpret_cast<char *>(p->work) + ws_layout(p->nchan, N).row);
    if (p->null_mode == PSS_NULL_DELAYED) {
        if (!p->inj_box) {
            k_box_row<<<stream_grid(N, 1), dim3(256), 0, st>>>(k, row);
            LAUNCHCHK();
            k.p.inj_box = row;
        } else {
            row = const_cast<float *>(p->inj_box);
        }
    }
    if (is_pow2(N) && N >= 64 && N <= 8192) return run_single(k, st);
    if (is_pow2(N) && N >= 16384 && N <= (1ll << 24)) return run_fourstep(k, st, row);
    if (smooth_split(N) && p->null_mode != PSS_NULL_DELAYED) return run_smooth(k, st);
    return run_fallback(k, st);
}


int pss_shift_rows(float *rows, int32_t nrows, int64_t n, int64_t ld, const uint64_t *ramp,
                   const float *nyq, void *work, void *stream) {
    if (n > 0 && (n & 1) && nrows > 0) {
        if (n > (1ll << 20)) return fail(PSS_EUNSUPPORTED, "odd-length shift_t above 2^20 samples (N=%lld)", (long long)n);
        if (ld < n) return fail(PSS_EINVAL, "ld < nsamp");
        return shift_rows_odd(rows, nrows, n, ld, ramp, work, (hipStream_t)stream);
    }
    PssPipeline p;
    memset(&p, 0, sizeof(p));
    p.nchan = nrows;
    p.nsamp = n;
    p.ld = ld;
    p.data = rows;
    p.work = work;
    p.src = PSS_SRC_LOAD;
    p.shift = 1;
    p.data_in_fft = 1;
    p.ramp = ramp;
    p.nyq_re = nyq;
    p.nyq_im = nyq;
    return pss_run(&p, stream);
}

int64_t pss_filter_workspace_bytes(int32_t nrows, int64_t n) {
    if (nrows <= 0 || n <= 0) return 0;
    return ws_layout(nrows, n, true).total;
}

int pss_filter_rows(float *rows, int32_t nrows, int64_t n, int64_t ld, const float *htab, void *work,
                    void *stream) {
    if (!htab) return fail(PSS_EINVAL, "filter_rows: htab is NULL");
    PssPipeline p;
    memset(&p, 0, sizeof(p));
    p.nchan = nrows;
    p.nsamp = n;
    p.ld = ld;
    p.data = rows;
    p.work = work;
    p.src = PSS_SRC_LOAD;
    p.shift = 1;
    p.data_in_fft = 1;
    p.htab = htab;
    return pss_run(&p, stream);
}

int pss_down_sample(const float *in, float *out, int32_t nrows, int64_t in_len, int64_t in_ld,
                    int32_t fact, void *stream) {
    if (fact < 1 || in_len % fact) return fail(PSS_EINVAL, "down_sample: %lld %% %d != 0", (long long)in_len, fact);
    if (nrows <= 0) return PSS_OK;
    if (!in || !out) return fail(PSS_EINVAL, "down_sample: NULL argument");
    if (in_ld < in_len) return fail(PSS_EINVAL, "down_sample: in_ld < in_len");
    if (nrows > 65535) return fail(PSS_EINVAL, "nchan %d > 65535 per launch", nrows);
    dim3 g = stream_grid(in_len / fact, nrows);
    hipLaunchKernelGGL(k_down_sample, g, dim3(256), 0, (hipStream_t)stream, in, out, in_len, in_ld, fact);
    LAUNCHCHK();
    return PSS_OK;
}

int pss_rebin(const float *in, float *out, int32_t nrows, int64_t in_len, int64_t in_ld, int32_t newlen,
              const int64_t *lo, const int64_t *hi, void *stream) {
    if (nrows <= 0 || newlen <= 0) return PSS_OK;
    // lo / hi are device arrays (the caller's windows, 0 <= lo_i <= hi_i <= in_len)
    if (!in || !out || !lo || !hi) return fail(PSS_EINVAL, "rebin: NULL argument");
    if (in_ld < in_len) return fail(PSS_EINVAL, "rebin: in_ld < in_len");
    if (nrows > 65535) return fail(PSS_EINVAL, "nchan %d > 65535 per launch", nrows);
    dim3 g = stream_grid(newlen, nrows);
    hipLaunchKernelGGL(k_rebin, g, dim3(256), 0, (hipStream_t)stream, in, out, in_ld, newlen, lo, hi);
    LAUNCHCHK();
    return PSS_OK;
}

int pss_clip_cast(const float *in, void *out, int64_t count, float clip, int32_t out_kind, void *stream) {
    if (out_kind != PSS_OUT_F32 && out_kind != PSS_OUT_I8) return fail(PSS_EINVAL, "out_kind");
    if (count <= 0) return PSS_OK;
    if (!in || !out) return fail(PSS_EINVAL, "clip_cast: NULL argument");
    dim3 g = stream_grid(count, 1);
    hipLaunchKernelGGL(k_clip_cast, g, dim3(256), 0, (hipStream_t)stream, in, out, count, clip, out_kind);
    LAUNCHCHK();
    return PSS_OK;
}

int pss_fold(const float *data, float *out, int32_t nchan, int64_t ld, int64_t npbins, int64_t n_fold,
             void *stream) {
    if (nchan <= 0 || npbins < 2 || n_fold < 0) return fail(PSS_EINVAL, "fold geometry");
    if (npbins + n_fold * (npbins / 2) > ld)
        return fail(PSS_EINVAL, "fold: %lld + %lld x %lld samples exceed the row (ld %lld)", (long long)npbins,
                    (long long)n_fold, (long long)(npbins / 2), (long long)ld);
    if (!data || !out || nchan > 65535) return fail(PSS_EINVAL, "fold: NULL argument or nchan > 65535");
    dim3 g = stream_grid(npbins / 2, nchan);
    hipLaunchKernelGGL(k_fold, g, dim3(256), 0, (hipStream_t)stream, data, out, ld, npbins, n_fold);
    LAUNCHCHK();
    return PSS_OK;
}

int pss_fold_periods(const float *data, float *out, int32_t nchan, int64_t ld, int64_t nbin, int64_t nper,
                     void *stream) {
    if (nchan <= 0 || nbin < 1 || nper < 1) return fail(PSS_EINVAL, "fold geometry");
    if (!data || !out || nchan > 65535) return fail(PSS_EINVAL, "fold: NULL argument or nchan > 65535");
    if (nper * nbin > ld) return fail(PSS_EINVAL, "fold: %lld periods of %lld bins exceed the row", (long long)nper,
                                      (long long)nbin);
    dim3 g = stream_grid(nbin, nchan);
    hipLaunchKernelGGL(k_fold_periods, g, dim3(256), 0, (hipStream_t)stream, data, out, ld, nbin, nper);
    LAUNCHCHK();
    return PSS_OK;
}

int pss_null_shift(const float *row, int64_t count, int64_t *out, void *stream) {
    if (!row || !out || count < 1) return fail(PSS_EINVAL, "null_shift: bad arguments");
    k_null_shift<<<1, 256, 0, (hipStream_t)stream>>>(row, count, out);
    LAUNCHCHK();
    return PSS_OK;
}

int pss_chi2_fill(float *out, int32_t nrows, int32_t chan0, int64_t n, float df, uint64_t seed,
                  uint32_t call_id, uint32_t purpose, void *stream) {
    if (nrows <= 0 || n <= 0) return PSS_OK;
    if (!out || nrows > 65535) return fail(PSS_EINVAL, "chi2_fill: NULL out or nrows > 65535");
    dim3 g = stream_grid((n + 3) / 4, nrows);
    hipLaunchKernelGGL(k_chi2_fill, g, dim3(256), 0, (hipStream_t)stream, out, n, chan0, df, seed,
                       call_id, purpose);
    LAUNCHCHK();
    return PSS_OK;
}

}  // extern "C"

