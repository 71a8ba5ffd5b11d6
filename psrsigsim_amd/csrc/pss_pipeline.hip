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

#include "pss_device.hpp"
#include "pss_fft.hpp"
#include "../../include/pss_hip.h"

// Fixed product choices (each measured against its alternatives, DESIGN.md
// sections 3 and 10; the rejected variants live in the git history):
//   * column blocks of the column passes mapped XCD-contiguously (xcd_block);
//   * 2^22 split 1024 x 4096 (rows of 4096 for 2^17 .. 2^22), 2^24 split
//     2048 x 8192;
//   * fast pass C on 16-column blocks of 1024 threads (C3), 16-column
//     register-resident blocks of 512 threads (C5, passC_fast32);
//   * the delayed-null mask table built on a side stream next to pass A, and
//     applied by the compacted fix-up (k_null_fix_list) after pass C.
static constexpr int kBC = 16, kTC = 1024;   // fast pass C block / threads (C3 and 2^17 .. 2^21)

using namespace pss;

// ---------------------------------------------------------------------------
// error reporting
// ---------------------------------------------------------------------------
static thread_local char g_err[512] = "";

static int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define HIPCHK(x)                                                              \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess)                                                  \
            return fail(PSS_EHIP, "%s: %s", #x, hipGetErrorString(e_));        \
    } while (0)

#define LAUNCHCHK()                                                            \
    do {                                                                       \
        hipError_t e_ = hipGetLastError();                                     \
        if (e_ != hipSuccess)                                                  \
            return fail(PSS_EHIP, "launch failed: %s", hipGetErrorString(e_)); \
    } while (0)

// ---------------------------------------------------------------------------
// opt-in per-kernel timing (bench.py): hipEvents recorded on the launch stream
// around every kernel of pss_run, summed per kernel kind on collect.
// ---------------------------------------------------------------------------
enum { TK_ELEM = 0, TK_SINGLE, TK_COLA, TK_ROW, TK_COLC, TK_FALLBACK, TK_NULLFIX, TK_N };
static bool g_timing = false;
struct TimedLaunch { int kind; int64_t units; hipEvent_t a, b; };
static TimedLaunch g_tl[4096];
static int g_ntl = 0;
static int g_tk_pending = -1;

static int64_t g_tk_units = 0;   // samples processed by the launch being timed

// (the events are created once per slot and reused: creating two events per
// launch inside the timed steps cost the host ~tens of microseconds each)
static void tk_begin(int kind, hipStream_t st) {
    if (!g_timing || g_ntl >= 4096) { g_tk_pending = -1; return; }
    TimedLaunch &t = g_tl[g_ntl];
    if (!t.a && hipEventCreate(&t.a) != hipSuccess) { t.a = nullptr; g_tk_pending = -1; return; }
    if (!t.b && hipEventCreate(&t.b) != hipSuccess) { t.b = nullptr; g_tk_pending = -1; return; }
    t.kind = kind;
    t.units = g_tk_units;
    (void)hipEventRecord(t.a, st);
    g_tk_pending = kind;
}
static void tk_end(hipStream_t st) {
    if (g_tk_pending < 0) return;
    (void)hipEventRecord(g_tl[g_ntl].b, st);
    ++g_ntl;
    g_tk_pending = -1;
}

// ---------------------------------------------------------------------------
// kernel parameters
// ---------------------------------------------------------------------------
struct KP {
    PssPipeline p;
    int64_t N;      // samples per row
    int64_t N1;     // four-step: column length (1 for single-pass)
    int64_t N2;     // four-step: row length    (N for single-pass)
    float invN;
    // four-step pair mode (two channels per complex row)
    int npairs;
    int poff;       // chan0 & 1: pairs are (even, odd) GLOBAL channels
    cf *Yd;         // data pair spill    [npairs][N1][sp]
    cf *Ym;         // node pair spill    [KCH/2][N1][N2] (mask table build)
    const cf *Mspec;// mask spectrum      [N1][N2] (natural k2 per row k1)
    // delayed-null mask table (four-step lengths; see k_mask_table)
    int mtab;               // 1: mask decisions come from the table
    int log2n;
    const uint2 *mt_bits;   // [N/32] {nulled-for-every-f bits, f-dependent bits}
    const uint32_t *mt_base;// [N/32] index of the word's first f-dependent position
    const float *mt_coef;   // [n_f_dependent][KCH] root records of the f-dependent positions (root_hit)
    const uint32_t *mbits;  // [nchan][N/32] per-channel null decisions (k_mask_bits)
    int mbB;                // column-block width B of pass C (mbits layout)
    const cf *rtab;         // [npairs][RFL][2] row-pass pair ramp factors {E, D} (k_pair_tab)
    hipEvent_t mask_ready;  // mask table built on a side stream: wait before its first use (or NULL)
    const uint32_t *wlist;  // delayed null: table words with a nulled position (any f)
    const uint32_t *nwlist; // its length (device)
};
// pair spill row pitch and per-pair stride (complex)
__host__ __device__ __forceinline__ int64_t rpitch(const KP &k) { return k.N2; }
__host__ __device__ __forceinline__ int64_t pstride(const KP &k) { return k.N1 * rpitch(k); }


// ---------------------------------------------------------------------------
// Delayed-null mask table.
//
// The reference shifts ONE box row (the same for every channel) by each
// channel's total delay s_c and nulls where the result exceeds 1
// (pulsar.py:306-330).  Write s = i + f (i integer, f in [0,1)).  For integer
// sample offsets d the shift_t kernel, Nyquist rule included, satisfies
// h_s(d) = h_f(d - i): the integer part is an exact circular roll, so
//     mask_c[n] = M(p, f_c),  p = (n - i_c) mod N,
// with M(p, f) = shift_t(box, f)[p] one function of (p, f) for all channels.
// As a function of f, M(p, .) is a trigonometric polynomial of bandwidth
// pi (bins |k| <= N/2), so a degree-11 Chebyshev interpolant in t = 2f - 1
// from KCH = 12 node shifts is exact to ~1e-9 relative (tools: DESIGN.md §3).
// Per position the table stores whether M > 1 for EVERY f (bound
// c0 -+ sum|c_n|), for NO f, or -- for the ~2% of positions near box edges
// where the answer depends on f -- the f values (as t) where the fp32
// interpolant crosses 1, found once per position by the table build
// (root_hit; the per-channel lookup is then two compares).  The node shifts are
// KCH/2 pair rows through the same FFT engine, once per run; per channel
// nothing but a table lookup remains (no per-channel mask FFT or spill).
// ---------------------------------------------------------------------------
static constexpr int KCH = 12;
// floats per f-dependent position record (root_hit): 16 (64 B, aligned)
static constexpr int KREC = 16;
// PCHIP intervals the fast pass A keeps in LDS (two rows; 69.7 KB FFT buffer +
// 12 KB still allows two 512-thread workgroups per CU).
static constexpr int kFastNint = 376;

// t = 2 f - 1 and i from the mask ramp word w = frac(s / N) 2^64 (N = 2^L)
__device__ __forceinline__ void mask_split(uint64_t w, int L, uint32_t &ishift, float &t) {
    ishift = (uint32_t)(w >> (64 - L));
    const uint64_t fr = w << L;                         // f in 2^-64 units
    t = fmaf((float)(uint32_t)(fr >> 40), 1.1920928955078125e-07f, -1.0f);   // 2 f - 1
}

// Clenshaw evaluation of the degree-11 Chebyshev interpolant at t (the mask
// value M(p, f), t = 2 f - 1), fp32: the table build's root scan uses it
__device__ __forceinline__ float cheb_eval_r(const float4 (&q)[3], float t) {
    const float4 a = q[0], b = q[1], d = q[2];
    const float cc[KCH] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, d.x, d.y, d.z, d.w};
    const float t2 = 2.0f * t;
    float b1 = 0.f, b2 = 0.f;
#pragma unroll
    for (int n = KCH - 1; n >= 1; --n) {
        const float b0 = fmaf(t2, b1, cc[n] - b2);
        b2 = b1;
        b1 = b0;
    }
    return fmaf(t, b1, cc[0] - b2);
}

// Decision of an f-dependent position from its ROOT record (k_mask_table):
// rec = {count, s0, r_1 .. r_10, -}: the fp32 Chebyshev value at t exceeds 1
// iff s0 XOR (the number of roots r_i < t) is odd.  The roots are where
// cheb_eval_r(c, .) > 1 flips, found by a 257-point scan of t in [-1, 1]
// (24 bisection steps per flip) whose cells are CERTIFIED to hold no hidden
// pair of flips (g = value - 1, D2 = max|g''| <= sum_n |c_n| n^2 (n^2 - 1) / 3
// by Markov's bound on T_n'', fp32 evaluation error included): a cell whose
// ends share a sign holds no root when min(|g(t_j)|, |g(t_j+1)|) > D2 h^2 / 8
// (the chord-interpolation error bound), and one with a sign change holds
// exactly one when the secant |g(t_j+1) - g(t_j)| / h exceeds D2 h (g' keeps
// its sign; ~2 % of the f-dependent positions of C3's mask fail this and keep
// coefficient records, measured with tools/mask_cert.py).  The rule then reproduces the direct
// evaluation except within ~1e-8 of a flip, with one 16-B load and two
// compares per position instead of 48 B of coefficients and a 12-term
// Clenshaw sum; unused roots are +inf.  A position whose cells cannot all be
// certified keeps its coefficients instead: rec = {-1, -, -, -, c_0 .. c_11},
// evaluated directly.  `a` is the record's first float4.
__device__ __forceinline__ bool root_hit(const float4 a, const float *rec, float t) {
    if (a.x < 0.f) {                     // uncertified: the coefficient record
        const float4 q[3] = {reinterpret_cast<const float4 *>(rec)[1], reinterpret_cast<const float4 *>(rec)[2],
                             reinterpret_cast<const float4 *>(rec)[3]};
        return cheb_eval_r(q, t) > 1.0f;
    }
    bool h = (a.y != 0.f) ^ (t > a.z) ^ (t > a.w);
    if (a.x > 2.f) {                    // rare: more than two flips over f in [0, 1)
        const float4 b = reinterpret_cast<const float4 *>(rec)[1], c = reinterpret_cast<const float4 *>(rec)[2];
        h ^= (t > b.x) ^ (t > b.y) ^ (t > b.z) ^ (t > b.w) ^ (t > c.x) ^ (t > c.y) ^ (t > c.z) ^ (t > c.w);
    }
    return h;
}

// Null decision bits (bit i: sample n0 + i) for 4 consecutive samples of a
// channel with mask split (ishift, t): a 4-bit window of the two table words
// covering positions p0..p0+3 (mod N), branch-free; the Chebyshev evaluation
// only where a position's decision depends on f (~2% of positions).
__device__ __forceinline__ uint32_t mask_hits4(const KP &k, int64_t n0, uint32_t ishift, float t) {
    const uint32_t nm = (uint32_t)k.N - 1u;
    const uint32_t p0 = ((uint32_t)n0 - ishift) & nm;
    const uint32_t w = p0 >> 5, w2 = (w + 1u) & (nm >> 5), sh = p0 & 31u;
    const uint2 A = k.mt_bits[w], Bw = k.mt_bits[w2];
    uint32_t r = (uint32_t)(((((uint64_t)Bw.x) << 32) | A.x) >> sh) & 15u;
    const uint32_t amb = (uint32_t)(((((uint64_t)Bw.y) << 32) | A.y) >> sh) & 15u;
    if (amb) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if ((amb >> i) & 1u) {
                const uint32_t p = (p0 + (uint32_t)i) & nm, pw = p >> 5;
                const uint32_t word = (pw == w) ? A.y : Bw.y;
                const uint32_t idx = k.mt_base[pw] + (uint32_t)__popc(word & ((1u << (p & 31u)) - 1u));
                const float *rec = k.mt_coef + (int64_t)idx * KREC;
                const bool hit = root_hit(reinterpret_cast<const float4 *>(rec)[0], rec, t);
                r = (r & ~(1u << i)) | ((uint32_t)hit << i);
            }
        }
    }
    return r;
}

// Null decisions of the RUN <= 32 contiguous samples n .. n + RUN - 1 of a
// channel with mask split (is, t): a window of the two table words covering
// them; the Chebyshev evaluation only at f-dependent positions (~2%).
__device__ __forceinline__ uint32_t mask_run(const KP &k, uint32_t n, uint32_t is, float t, uint32_t RUN) {
    const uint32_t nm = (uint32_t)k.N - 1u, wm = nm >> 5;
    const uint32_t p0 = (n - is) & nm, w = p0 >> 5, w2 = (w + 1u) & wm, sh = p0 & 31u;
    const uint2 A = k.mt_bits[w], Bw = k.mt_bits[w2];
    const uint32_t msk = RUN >= 32u ? 0xffffffffu : ((1u << RUN) - 1u);
    uint32_t r32 = (uint32_t)(((((uint64_t)Bw.x) << 32) | A.x) >> sh) & msk;
    uint32_t amb = (uint32_t)(((((uint64_t)Bw.y) << 32) | A.y) >> sh) & msk;
    if (!amb) return r32;
    // Ambiguous positions cluster at pulse edges (a lane may hold ~20): take
    // them four at a time so the coefficient loads of a group are in flight
    // together instead of one exposed latency per position (the table bases
    // of the two words are loaded once).
    const uint32_t baseA = k.mt_base[w], baseB = k.mt_base[w2];
    while (amb) {
        uint32_t ii[4], idx[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            ii[u] = amb ? (uint32_t)__ffs(amb) - 1u : 32u;
            amb &= amb - 1u;
            const uint32_t p = (p0 + (ii[u] & 31u)) & nm;
            const bool inA = (p >> 5) == w;
            const uint32_t word = inA ? A.y : Bw.y;
            idx[u] = (inA ? baseA : baseB) + (uint32_t)__popc(word & ((1u << (p & 31u)) - 1u));
        }
        float4 a[4];
        const float *rec[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            rec[u] = k.mt_coef + (int64_t)(ii[u] < 32u ? idx[u] : idx[0]) * KREC;
            a[u] = reinterpret_cast<const float4 *>(rec[u])[0];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (ii[u] < 32u) {
                const bool hit = root_hit(a[u], rec[u], t);
                r32 = (r32 & ~(1u << ii[u])) | ((uint32_t)hit << ii[u]);
            }
        }
    }
    return r32;
}

// Per-channel null decisions for the four-step column pass C.  A pass-C
// workgroup owns the B columns [n20, n20 + B) of every row n1 (samples
// n1 N2 + n20 + b); looking the table up there means scattered loads 8192
// samples apart.  k_mask_bits resolves the table once per channel into one bit
// per sample, laid out in pass-C order: entry (n20 / B, n1) holds B bits
// (B % 4 == 0), entries in a bit stream [chan][N2 / B][N1][B], so a workgroup
// reads its decisions as one contiguous N1 * B-bit run per channel.
__global__ __launch_bounds__(256) void k_mask_bits(KP k, uint32_t *bm) {
    const int r = blockIdx.y;
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;          // output word of channel r
    const uint32_t wm = ((uint32_t)k.N - 1u) >> 5;
    if (j > wm) return;
    uint32_t is;
    float t;
    mask_split((uint64_t)k.p.mask_ramp[r], k.log2n, is, t);
    const uint32_t B = (uint32_t)k.mbB, RUN = B < 32u ? B : 32u;
    const uint32_t N1 = (uint32_t)k.N1, N2 = (uint32_t)k.N2;
    uint32_t out = 0;
    for (uint32_t s = 0; s < 32u; s += RUN) {          // runs of RUN contiguous samples
        const uint32_t bp = (j << 5) + s, e = bp / B, b = bp - e * B;
        const uint32_t n = (e % N1) * N2 + (e / N1) * B + b;
        out |= mask_run(k, n, is, t, RUN) << s;
    }
    bm[(int64_t)r * (wm + 1u) + j] = out;
}

// Table words (32 positions each) that hold a position nulled for some f:
// the only words the null fix-up has to visit (the nulled pulses and their
// Gibbs ringing, ~10-20% of the row).  Compacted once per run.
__global__ __launch_bounds__(256) void k_mask_words(const uint2 *bits, uint32_t nwords, uint32_t *list,
                                                    uint32_t *count) {
    const uint32_t w = blockIdx.x * 256u + threadIdx.x;
    bool nz = false;
    if (w < nwords) {
        const uint2 b = bits[w];
        nz = (b.x | b.y) != 0u;
    }
    const uint64_t bal = __ballot(nz);
    const int lane = threadIdx.x & 63;
    uint32_t b0 = 0;
    if (lane == 0 && bal) b0 = atomicAdd(count, (uint32_t)__popcll(bal));
    b0 = __shfl(b0, 0);
    if (nz) list[b0 + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = w;
}

// Delayed null fix-up driven by the word list: item (channel r, listed table
// word w) covers data samples (32 w + i_c + j) mod N, j < 32 (the channel's
// integer shift i_c carries table position p to sample p + i_c); the nulled
// ones are rewritten as replacement + noise with the same Philox draws and
// expression as epilogue4 (bitwise the generic kernels' values).  A sample
// belongs to exactly one item, so items write disjoint samples; 4-sample
// groups cut by an unaligned window are drawn by both neighbours, each
// writing its own samples.  Grid-stride over the list (its length is only
// known on the device).
__global__ __launch_bounds__(256) void k_null_fix_list(KP k) {
    __shared__ uint32_t desc[4][64 * 9];
    __shared__ uint32_t dbase[4][64 * 9];
    const int r = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const PssPipeline &p = k.p;
    const uint32_t nl = *k.nwlist;
    const uint32_t nm = (uint32_t)k.N - 1u;
    uint32_t is;
    float t;
    mask_split((uint64_t)p.mask_ramp[r], k.log2n, is, t);
    const uint32_t c = (uint32_t)(p.chan0 + r);
    float *row = p.data + (int64_t)r * p.ld;
    const Rng gn(p.seed, p.call_noise, P_NOISE), gr(p.seed, p.call_null, P_REP);
    const float nn = p.noise_norm, sc = p.null_rep_scale;
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t i0 = blockIdx.x * 256u; i0 < nl; i0 += stride) {       // wave-uniform trip count
        const uint32_t i = i0 + threadIdx.x;
        uint32_t hits = 0, n0 = 0;
        if (i < nl) {
            const uint32_t w = k.wlist[i];
            n0 = ((w << 5) + is) & nm;                   // data sample of table position 32 w
            hits = mask_run(k, n0, is, t, 32u);
        }
        if (__ballot(hits != 0u) == 0ull) continue;
        // (group, 4-bit mask) entries of this lane: samples n0 + j in groups
        // of 4 aligned DATA indices (the Philox block of sample n is n >> 2).
        // Entries are listed lane-major (a lane's groups consecutive), so the
        // lanes of the drawing loop below store consecutive 16-B groups of
        // one word -- whole 128-B lines -- instead of one group of each of 64
        // words per store instruction.  The exclusive prefix of the per-lane
        // group counts (< 16) comes from four ballots.
        const uint32_t a = n0 & 3u;                      // offset of n0 in its group
        const uint64_t hx = (uint64_t)hits << a;         // hit bits by position in the aligned span
        uint32_t cnt = 0;
#pragma unroll
        for (int g = 0; g < 9; ++g) cnt += ((uint32_t)(hx >> (4 * g)) & 15u) ? 1u : 0u;
        const uint64_t below = (1ull << lane) - 1ull;
        uint32_t e = 0, total = 0;
#pragma unroll
        for (int bit = 0; bit < 4; ++bit) {
            const uint64_t bal = __ballot((cnt >> bit) & 1u);
            e += (uint32_t)__popcll(bal & below) << bit;
            total += (uint32_t)__popcll(bal) << bit;
        }
#pragma unroll
        for (int g = 0; g < 9; ++g) {
            const uint32_t h = (uint32_t)(hx >> (4 * g)) & 15u;
            if (h) {
                desc[wv][e] = h;
                dbase[wv][e] = ((n0 - a) + 4u * (uint32_t)g) & nm;   // first sample of the group
                ++e;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t e = (uint32_t)lane; e < total; e += 64u) {
            const uint32_t h = desc[wv][e], nb = dbase[wv][e];
            PSS_DASSERT((int64_t)nb + 4 <= k.N && (nb & 3u) == 0u);
            const float4 xn = chi2_1x4(gn.bits(nb >> 2, c, 0u));
            const float4 xr = chi2_1x4(gr.bits(nb >> 2, c, 0u));
            const float vn[4] = {xn.x, xn.y, xn.z, xn.w}, vr[4] = {xr.x, xr.y, xr.z, xr.w};
            if (h == 15u) {
                *reinterpret_cast<float4 *>(row + nb) =
                    make_float4(fmaf(nn, vn[0], vr[0] * sc), fmaf(nn, vn[1], vr[1] * sc),
                                fmaf(nn, vn[2], vr[2] * sc), fmaf(nn, vn[3], vr[3] * sc));
                continue;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if ((h >> q) & 1u) row[nb + q] = fmaf(nn, vn[q], vr[q] * sc);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// 4 null decisions of channel row r for samples n1 N2 + n20 + b4 .. + 3.
// (column block blockIdx.x of B columns, N1 rows; B, N1 as in pass C)
template <int B, int N1>
__device__ __forceinline__ uint32_t mask_bits4(const KP &k, int r, int cbx, int n1, int b4) {
    const uint32_t bp = (((uint32_t)cbx * (uint32_t)N1 + (uint32_t)n1) * (uint32_t)B) + (uint32_t)b4;
    return (k.mbits[(int64_t)r * (k.N >> 5) + (bp >> 5)] >> (bp & 31u)) & 15u;
}

// XCD-aware block order of the column passes.  Workgroups are dispatched
// round-robin over the 8 XCDs (linear id % 8), each with its own L2; the
// passes touch B-column segments of every row (32 B of fp32 output per channel
// for B = 8, a quarter of a 128-B line).  Remapping linear id ->
// (id % 8) * (total / 8) + id / 8 gives each XCD a contiguous range of column
// blocks, so the pieces of a line are written through the same L2 at about the
// same time and merge there.  Measured (pass C, 2048 x 2^22): 17.8-19 ms with
// the remap, 61 ms without, 58 ms with the blocks bit-reversed over the row;
// contiguous (wrong-place) stores would take 14.3 ms -- the residual cost of
// the strided output is ~4 ms.  Non-temporal / sc1 loads of the spill make it
// worse (21-25 ms): neighbouring blocks share the spill's lines through L2.
// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

__device__ __forceinline__ void xcd_block(int &bx, int &by) {
    const uint32_t gx = gridDim.x, total = gx * gridDim.y;
    const uint32_t id = blockIdx.x + blockIdx.y * gx;
    const uint32_t l = ((total & 7u) == 0u) ? (id & 7u) * (total >> 3) + (id >> 3) : id;
    by = (int)(l / gx);
    bx = (int)(l - (uint32_t)by * gx);
}

__device__ __forceinline__ int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}

// Box (nulled pulse) covering sample n, following the reference's numpy
// indexing: bins = arange(Nph p, Nph (p+1)) + shift_val, filtered < N; negative
// bins address from the end; later pulses in the choice list overwrite.
__device__ __forceinline__ bool box_of(const KP &k, int64_t n, int &rank, int &j) {
    const PssPipeline &p = k.p;
    rank = -1;
    const int64_t nph = p.nph;
    const int64_t shift = p.null_shift_dev ? *p.null_shift_dev : p.null_shift;
    int64_t q = n - shift;
    int64_t s = floordiv(q, nph);
    if (s >= 0 && s < p.null_slots) {
        int r = p.null_rank[s];
        if (r >= 0) { rank = r; j = (int)(q - s * nph); }
    }
    q = n - k.N - shift;                 // the same sample reached by a negative bin
    s = floordiv(q, nph);
    if (s >= 0 && s < p.null_slots) {
        int r = p.null_rank[s];
        if (r > rank) { rank = r; j = (int)(q - s * nph); }
    }
    return rank >= 0;
}

__device__ __forceinline__ float box_value(const KP &k, int64_t n, int rank, int j) {
    const PssPipeline &p = k.p;
    if (p.inj_box) return p.inj_box[n];
    Rng g(p.seed, p.call_null, P_BOX);
    return chi2_general(g, (uint32_t)j, (uint32_t)rank, p.null_box_df) * p.null_box_scale;
}

// chi2 draws for 4 consecutive samples n0..n0+3 (n0 % 4 == 0) of channel c.
// df == 1: one Philox block per 4 samples; otherwise the Marsaglia-Tsang
// pair sampler, one shared block per 2 samples (chi2_pair).
__device__ __forceinline__ void draw4(const Rng &g, int64_t n0, uint32_t c, float df, float (&x)[4]) {
    if (df == 1.0f) {
        float4 q = chi2_1x4(g.bits((uint32_t)(n0 >> 2), c, (uint32_t)(n0 >> 34)));
        x[0] = q.x; x[1] = q.y; x[2] = q.z; x[3] = q.w;
    } else {
        const uint32_t m = (uint32_t)(n0 >> 1);
        chi2_pair(g, m, c, df, x[0], x[1]);
        chi2_pair(g, m + 1u, c, df, x[2], x[3]);
    }
}

// Interval index and fraction of sample n's pulse phase (shared by every
// channel: only the coefficient row differs).
__device__ __forceinline__ void pchip_locate(const KP &k, int64_t n, uint32_t &iv, float &u) {
    const PssPipeline &p = k.p;
    // ph = n * phase_step mod 2^64 (2^-64 cycles), n < 2^32: 32-bit products only
    const uint32_t nn = (uint32_t)n;
    const uint64_t ph = (uint64_t)nn * (uint32_t)p.phase_step +
                        ((uint64_t)(nn * (uint32_t)(p.phase_step >> 32)) << 32);
    // ph * M = iv 2^64 + fraction; u = (ph * M) >> 32 holds iv and fraction bits 32..63
    const uint64_t t = (uint64_t)(uint32_t)ph * p.knot_m;
    const uint64_t u64 = (uint64_t)(uint32_t)(ph >> 32) * p.knot_m + (t >> 32);
    iv = (uint32_t)(u64 >> 32);                                    // interval index
    u = frac23((uint32_t)u64);                                     // fraction, 23 bits
    if (iv >= (uint32_t)p.nint) {                                  // extrapolate
        u += (float)(iv - (uint32_t)(p.nint - 1));
        iv = p.nint - 1;
    }
}

// The same (interval, fraction) for consecutive samples by increments: the
// 96-bit product A(n) = (n phase_step mod 2^64) * knot_m, kept as three
// 32-bit words (hi = interval field, mid = fraction, lo = guard), advances by
// D = phase_step * knot_m; when the phase wraps the interval field comes back
// by knot_m.  Exact integer arithmetic: bitwise the values pchip_locate
// computes, at one add-with-carry chain and a min per sample (the 64-bit form
// compiled to nine VALU per step) instead of four 32 x 32 -> 64 multiplies.
struct PhaseWalk {
    uint32_t lo, mid, hi;
    __device__ __forceinline__ void start(const PssPipeline &p, uint32_t n) {
        const uint64_t ph = (uint64_t)n * (uint32_t)p.phase_step + ((uint64_t)(n * (uint32_t)(p.phase_step >> 32)) << 32);
        const uint64_t t = (uint64_t)(uint32_t)ph * p.knot_m;
        lo = (uint32_t)t;
        const uint64_t u64 = (uint64_t)(uint32_t)(ph >> 32) * p.knot_m + (t >> 32);
        mid = (uint32_t)u64;
        hi = (uint32_t)(u64 >> 32);
    }
    __device__ __forceinline__ void step(uint32_t dlo, uint64_t dhi, uint32_t M) {
        unsigned c;
        lo = __builtin_addc(lo, dlo, 0u, &c);
        mid = __builtin_addc(mid, (uint32_t)dhi, c, &c);
        hi = hi + (uint32_t)(dhi >> 32) + c;
        // (hi >= M) ? hi - M : hi -- hi < 2 M here, and for hi < M the
        // difference wraps above hi (M <= 2^31)
        hi = min(hi, hi - M);
    }
    __device__ __forceinline__ void get(const PssPipeline &p, uint32_t &iv, float &u) const {
        iv = hi;
        u = frac23(mid);
        if (iv >= (uint32_t)p.nint) {
            u += (float)(iv - (uint32_t)(p.nint - 1));
            iv = p.nint - 1;
        }
    }
    // the same for a table that spans the whole period (nint == knot_m, the
    // host's extrapolated pieces appended: pulsar._device_table), where
    // iv < knot_m needs no clamp -- bitwise what get() returns then
    __device__ __forceinline__ void get_full(uint32_t &iv, float &u) const {
        iv = hi;
        u = frac23(mid);
    }
};
__device__ __forceinline__ void phase_delta(const PssPipeline &p, uint32_t &dlo, uint64_t &dhi) {
    const uint64_t t = (uint64_t)(uint32_t)p.phase_step * p.knot_m;
    dlo = (uint32_t)t;
    dhi = (uint64_t)(uint32_t)(p.phase_step >> 32) * p.knot_m + (t >> 32);
}
// ... for a walk in strides of S samples: D = (S phase_step mod 2^64) knot_m
// (exact: the walk's sum stays below 2 knot_m in the interval field)
__device__ __forceinline__ void phase_delta_n(const PssPipeline &p, uint64_t S, uint32_t &dlo, uint64_t &dhi) {
    const uint64_t ps = p.phase_step * S;
    const uint64_t t = (uint64_t)(uint32_t)ps * p.knot_m;
    dlo = (uint32_t)t;
    dhi = (uint64_t)(uint32_t)(ps >> 32) * p.knot_m + (t >> 32);
}

__device__ __forceinline__ float pchip_row(const KP &k, int prow, uint32_t iv, float u) {
    float4 cc;
    if (k.p.prof_split) {
        // non-uniform knots: cell iv holds the cubics on either side of its
        // one interior knot (both in the cell coordinate u)
        const float4 *c = reinterpret_cast<const float4 *>(k.p.prof) + ((int64_t)prow * k.p.nint + iv) * 2;
        const float s = k.p.prof[(int64_t)k.p.prof_rows * k.p.nint * 8 + iv];
        cc = (u >= s) ? c[1] : c[0];
    } else {
        cc = reinterpret_cast<const float4 *>(k.p.prof)[(int64_t)prow * k.p.nint + iv];
    }
    return fmaf(fmaf(fmaf(cc.x, u, cc.y), u, cc.z), u, cc.w);
}

__device__ __forceinline__ float pchip_eval(const KP &k, int prow, int64_t n) {
    uint32_t iv;
    float u;
    pchip_locate(k, n, iv, u);
    return pchip_row(k, prow, iv, u);
}

// Analytic Gaussian portrait at sample n's pulse phase (amplitude pulses of
// a GaussProfile / 1-D GaussPortrait, portraits.py:143-178, 277-290):
// prof = [nint components][4] = {peak, 1/width, amp/Amax, 0}, channel
// independent; the phase is pchip_locate's fraction with knot_m = 1.
__device__ __forceinline__ float gauss_eval(const KP &k, int64_t n) {
    uint32_t iv;
    float u;
    pchip_locate(k, n, iv, u);
    const float4 *cp = reinterpret_cast<const float4 *>(k.p.prof);
    float acc = 0.f;
    for (int j = 0; j < k.p.nint; ++j) {
        const float4 c = cp[j];
        const float d = (u - c.x) * c.y;
        acc = fmaf(c.z, __expf(-0.5f * d * d), acc);
    }
    return acc;
}

// Source stage for 4 consecutive samples (cnt valid) of local row r.
// re = data (generated or loaded, with an undelayed null applied);
// im = delayed-null box mask (0 elsewhere).
__device__ __forceinline__ void source4(const KP &k, int r, int64_t n0, int cnt,
                                        float (&re)[4], float (&im)[4], bool want_re,
                                        bool want_im = true) {
    const PssPipeline &p = k.p;
    const uint32_t c = (uint32_t)(p.chan0 + r);
    PSS_DASSERT(r >= 0 && r < p.nchan && n0 >= 0 && n0 + cnt <= k.N);
#pragma unroll
    for (int i = 0; i < 4; ++i) { re[i] = 0.f; im[i] = 0.f; }
    if (want_re) {
        if (p.src == PSS_SRC_LOAD) {
            const float *row = p.data + (int64_t)r * p.ld;
#pragma unroll
            for (int i = 0; i < 4; ++i) if (i < cnt) re[i] = row[n0 + i];
        } else {
            float x[4];
            float dn = p.draw_norm;
            if (p.inj_gen) {
                const float *row = p.inj_gen + (int64_t)r * k.N;
#pragma unroll
                for (int i = 0; i < 4; ++i) x[i] = (i < cnt) ? row[n0 + i] : 0.f;
            } else if (p.gen_amp) {
                Rng g(p.seed, p.call_gen, P_PULSE);
                const float4 z = normal_x4(g.bits((uint32_t)(n0 >> 2), c, (uint32_t)(n0 >> 34)));
                x[0] = z.x; x[1] = z.y; x[2] = z.z; x[3] = z.w;
            } else if (p.gen_df == 1.0f) {
                // chi2(1) draws with draw_norm folded into the sampler (as the
                // fast pass A draws them: bitwise the same values)
                // (Philox block n >> 2 holds samples 4 (n >> 2) .. + 3 at every N)
                Rng g(p.seed, p.call_gen, P_PULSE);
                const float4 q = chi2_1x4(g.bits((uint32_t)(n0 >> 2), c, (uint32_t)(n0 >> 34)), p.draw_norm);
                x[0] = q.x; x[1] = q.y; x[2] = q.z; x[3] = q.w;
                dn = 1.0f;                                   // (x * 1 is exact)
            } else {
                Rng g(p.seed, p.call_gen, P_PULSE);
                draw4(g, n0, c, p.gen_df, x);
            }
            const int prow = (p.prof_rows == 1) ? 0 : (int)c - p.prof_row0;
            if (p.src == PSS_SRC_SEARCH && p.gen_amp) {
                // amplitude pulses: sqrt(calc_profiles(phase)) x N(0, 1)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (i < cnt) {
                        const float pr = (p.gen_amp == 2) ? gauss_eval(k, n0 + i) : pchip_eval(k, prow, n0 + i);
                        re[i] = sqrtf(fmaxf(pr, 0.0f)) * x[i] * dn;
                    }
                }
            } else if (p.src == PSS_SRC_SEARCH) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (i < cnt) re[i] = pchip_eval(k, prow, n0 + i) * x[i] * dn;
            } else {   // FOLD
                const float *pr = p.prof + (int64_t)prow * p.nph;
                uint32_t b = (uint32_t)(n0 % p.nph);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (i < cnt) re[i] = pr[b] * x[i] * dn;
                    if (++b == (uint32_t)p.nph) b = 0;
                }
            }
        }
        if (p.null_mode == PSS_NULL_UNDELAYED) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int rk, j;
                if (i < cnt && box_of(k, n0 + i, rk, j)) re[i] = box_value(k, n0 + i, rk, j);
            }
        }
    }
    if (want_im && p.null_mode == PSS_NULL_DELAYED) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int rk, j;
            if (i < cnt) {
                if (p.inj_box) im[i] = p.inj_box[n0 + i];
                else if (box_of(k, n0 + i, rk, j)) im[i] = box_value(k, n0 + i, rk, j);
            }
        }
    }
}

// observe()'s resampled pre-noise copy (PssPipeline.out_len > 0): the
// samples n0 .. n0 + cnt - 1 of row r added into the float64 sums of the
// windows [lo_j, hi_j) that hold them (down_sample, utils.py:62-68: lo_j =
// j f; rebin, utils.py:71-91: lo_j = ceil(j step), hi_j = ceil(j step + step)
// clipped to N, so neighbouring windows may share a sample).  The edges are
// recomputed from step with the host's float64 operations (out_lo / out_hi
// serve the finalize kernel's counts); a window holding n is floor(n / step)
// or the one before.  A lane's samples form a head piece (its first window)
// and a tail piece (its last; pieces in between go straight to their
// atomics); the head joins the previous lane's tail when they are the same
// window, and the tails are summed over each run of lanes with the same
// window -- a segmented reduction by doubling that only extends a sum over
// lanes it has covered without a gap, and stops once no run is still
// growing -- so one no-return float64 atomic leaves the wave per window
// piece.  (Within-wave sums in fp32: at most 256 samples, summed as a tree.)
// Waves whose lanes hold different rows (the single-workgroup kernel's row
// batches) skip the cross-lane step.  k_out_finalize divides, clips and casts
// (telescope.py:140-145).  All active lanes of a wave call it together (the
// epilogues' item loops are wave-uniform up to their tails; inactive lanes
// are masked out through the ballot).
__device__ __forceinline__ void out_windows(const PssPipeline &p, int r, uint32_t N, uint32_t n0, int cnt,
                                            const float (&v)[4]) {
    const int lane = (int)__lane_id();
    const uint64_t act = __ballot(1);
    const uint32_t L = (uint32_t)p.out_len;
    const bool uniform = p.out_lo == nullptr;
    const double step = p.out_step;
    const uint32_t f = (uint32_t)step;
    double *acc = p.out_acc + (int64_t)r * L;
    const uint32_t last = n0 + (uint32_t)cnt - 1u;
    int64_t ja, jb;
    if (uniform) {
        ja = n0 / f;
        jb = last / f;
    } else {
        const double inv = 1.0 / step;      // (wave-uniform: hoisted by the compiler)
        ja = (int64_t)floor((double)n0 * inv) - 2;
        jb = (int64_t)floor((double)last * inv) + 1;
    }
    ja = ja < 0 ? 0 : ja;
    jb = jb > (int64_t)L - 1 ? (int64_t)L - 1 : jb;
    uint32_t jH = 0xffffffffu, jT = 0xffffffffu;      // head / tail window, ~0: none
    float sH = 0.f, sT = 0.f;
    for (int64_t jj = ja; jj <= jb; ++jj) {
        const uint32_t j = (uint32_t)jj;
        uint32_t lo, hi;
        if (uniform) {
            lo = j * f;
            hi = lo + f;
        } else {
            // two statements: the sum is not contracted into an fma
            const double lb = (double)j * step;
            const double rb = lb + step;
            lo = (uint32_t)ceil(lb);
            hi = (uint32_t)ceil(rb);
            hi = hi > N ? N : hi;
        }
        float s = 0.f;
        bool any = false;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t n = n0 + (uint32_t)i;
            if (i < cnt && n >= lo && n < hi) {
                s += v[i];
                any = true;
            }
        }
        if (!any) continue;
        if (jT == 0xffffffffu) {
            jH = jT = j;
            sT = s;
        } else {
            if (jH == jT) sH = sT;                            // the first window becomes the head
            else unsafeAtomicAdd(acc + jT, (double)sT);        // a window in the middle of the lane
            jT = j;
            sT = s;
        }
    }
    const bool has_head = jT != 0xffffffffu && jH != jT;
    const int r0 = __builtin_amdgcn_readfirstlane(r);
    if (__ballot(r != r0) != 0ull) {
        // lanes of several rows: no cross-lane merge
        if (has_head) unsafeAtomicAdd(acc + jH, (double)sH);
        if (jT != 0xffffffffu) unsafeAtomicAdd(acc + jT, (double)sT);
        return;
    }
    // the head joins the previous lane's tail (the same window)
    const uint32_t nxt_h = (uint32_t)__shfl_down((int)(has_head ? jH : 0xffffffffu), 1);
    const float nxt_s = __shfl_down(sH, 1);
    const uint32_t prv_t = (uint32_t)__shfl_up((int)jT, 1);
    const bool nxt_ok = lane < 63 && ((act >> (lane + 1)) & 1ull);
    const bool prv_ok = lane > 0 && ((act >> (lane - 1)) & 1ull);
    if (jT != 0xffffffffu && nxt_ok && nxt_h == jT) sT += nxt_s;
    if (has_head && !(prv_ok && prv_t == jH)) unsafeAtomicAdd(acc + jH, (double)sH);
    // segmented sum of the tails over runs of lanes with one window
    const uint32_t key = jT != 0xffffffffu ? jT : 0x80000000u + (uint32_t)lane;   // no tail: a key of its own
    float sum = sT;
    int len = 1;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t ok_ = (uint32_t)__shfl_down((int)key, d);
        const bool grow = len == d && lane + d < 64 && ((act >> (lane + d)) & 1ull) && ok_ == key;
        if (__ballot(grow) == 0ull) break;
        const float os = __shfl_down(sum, d);
        const int ol = __shfl_down(len, d);
        if (grow) {
            sum += os;
            len += ol;
        }
    }
    if (jT != 0xffffffffu && !(prv_ok && prv_t == key)) unsafeAtomicAdd(acc + jT, (double)sum);
}

// Epilogue for 4 consecutive samples: delayed-null replacement where the
// shifted mask exceeds 1, the observe() pre-noise copy, radiometer noise, store.
// `pre` holds the data value (FFT output already scaled by 1/N, or the source).
__device__ __forceinline__ void epilogue4(const KP &k, int r, int64_t n0, int cnt,
                                          float (&pre)[4], const float (&mask)[4], bool load_data) {
    const PssPipeline &p = k.p;
    const uint32_t c = (uint32_t)(p.chan0 + r);
    float *row = p.data + (int64_t)r * p.ld;
    PSS_DASSERT(r >= 0 && r < p.nchan && n0 >= 0 && n0 + cnt <= k.N);
    if (load_data) {
#pragma unroll
        for (int i = 0; i < 4; ++i) if (i < cnt) pre[i] = row[n0 + i];
    }
    if (p.null_mode == PSS_NULL_DELAYED) {
        const bool any = (mask[0] > 1.0f) | (mask[1] > 1.0f) | (mask[2] > 1.0f) | (mask[3] > 1.0f);
        if (any) {
            float x[4];
            if (p.inj_rep) {
#pragma unroll
                for (int i = 0; i < 4; ++i) x[i] = (i < cnt) ? p.inj_rep[(int64_t)r * k.N + n0 + i] : 0.f;
            } else {
                Rng g(p.seed, p.call_null, P_REP);
                draw4(g, n0, c, p.null_rep_df, x);
#pragma unroll
                for (int i = 0; i < 4; ++i) x[i] *= p.null_rep_scale;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (i < cnt && mask[i] > 1.0f) pre[i] = x[i];
        }
    }
    if (p.out_kind != PSS_OUT_NONE && p.out_len > 0) {
        out_windows(p, r, (uint32_t)k.N, (uint32_t)n0, cnt, pre);
    } else if (p.out_kind == PSS_OUT_F32) {
        float *o = (float *)p.out + (int64_t)r * k.N;
#pragma unroll
        for (int i = 0; i < 4; ++i) if (i < cnt) o[n0 + i] = (pre[i] > p.clip) ? p.clip : pre[i];
    } else if (p.out_kind == PSS_OUT_I8) {
        int8_t *o = (int8_t *)p.out + (int64_t)r * k.N;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i < cnt) {
                float v = (pre[i] > p.clip) ? p.clip : pre[i];
                v = fminf(fmaxf(v, -128.f), 127.f);
                o[n0 + i] = (int8_t)(int)truncf(v);
            }
        }
    }
    if (p.noise) {
        float x[4];
        if (p.inj_noise) {
            const float *nr = p.inj_noise + (int64_t)r * k.N;
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = (i < cnt) ? nr[n0 + i] : 0.f;
        } else {
            Rng g(p.seed, p.call_noise, P_NOISE);
            draw4(g, n0, c, p.noise_df, x);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) pre[i] = fmaf(p.noise_norm, x[i], pre[i]);
    }
    if (cnt == 4 && (((uintptr_t)(row + n0)) & 15) == 0) {
        *reinterpret_cast<float4 *>(row + n0) = make_float4(pre[0], pre[1], pre[2], pre[3]);
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) if (i < cnt) row[n0 + i] = pre[i];
    }
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

__device__ __forceinline__ cf apply_ramp_delay(const KP &k, int r, int64_t kb, cf z);

// Scattering-tail transfer function of row r at bin kb (extension, see
// PssPipeline.tail_a): H = (1 - a) / (1 - a e^{-2 pi i kb/N}); exactly 1 at DC
// and real (1-a)/(1+a) at Nyquist, Hermitian in kb, so irfft stays real.
__device__ __forceinline__ cf tail_factor(float a, cf w) {
    // w = e^{-2 pi i kb / N}; 1/(1 - a w) = conj(d) / |d|^2, d = 1 - a w
    const float dr = fmaf(-a, w.x, 1.0f), di = -a * w.y;
    const float s = (1.0f - a) / fmaf(dr, dr, di * di);
    return make_float2(dr * s, -di * s);
}
__device__ __forceinline__ cf bin_phasor(int64_t kb, int64_t N) {
    const int64_t kk = (2 * kb > N) ? kb - N : kb;
    return expi_rev(-(float)((double)kk / (double)N));
}

// exp(-2 pi i k' s / N) for frequency bin k, with the reference's Nyquist
// rule applied separately to the real (data) and imaginary (mask) parts.
__device__ __forceinline__ cf apply_ramp(const KP &k, int r, int64_t kb, cf z) {
    if (k.p.tail_a && !k.p.htab) {
        const cf h = tail_factor(k.p.tail_a[r], bin_phasor(kb, k.N));
        const cf t = apply_ramp_delay(k, r, kb, z);
        if (kb == 0 || 2 * kb == k.N) return make_float2(t.x * h.x, t.y * h.x);   // real parts only
        return cmul(t, h);
    }
    return apply_ramp_delay(k, r, kb, z);
}
__device__ __forceinline__ cf apply_ramp_delay(const KP &k, int r, int64_t kb, cf z) {
    const PssPipeline &p = k.p;
    const int64_t N = k.N;
    if (p.htab) {
        // per-bin transfer function of the rfft bins; Hermitian extension,
        // DC and Nyquist keep Re H only (irfft drops their imaginary parts)
        const bool upper = 2 * kb > N;
        const cf h = reinterpret_cast<const cf *>(p.htab)[upper ? N - kb : kb];
        if (kb == 0 || 2 * kb == N) return make_float2(z.x * h.x, z.y * h.x);
        return cmul(z, make_float2(h.x, upper ? -h.y : h.y));
    }
    if (2 * kb == N) return make_float2(z.x * p.nyq_re[r], z.y * p.nyq_im[r]);
    if (kb == 0) return z;
    const int64_t kk = (2 * kb > N) ? kb - N : kb;
    const uint64_t ph = (uint64_t)kk * p.ramp[r];
    return cmul(z, expi_rev(-fix_to_rev(ph)));
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

// ---------------------------------------------------------------------------
// path 1: whole row(s) in LDS.  BATCH rows of length L per workgroup.
// ---------------------------------------------------------------------------
template <int L, int BATCH, int T, typename FWD, typename INV>
struct SinglePass;

template <int L, int BATCH, int T, int... F, int... I>
struct SinglePass<L, BATCH, T, RList<F...>, RList<I...>> {
    using FF = Fft<L, BATCH, T>;
    static constexpr int E = FF::E;
    static constexpr int RF0 = FF::template first<F...>();
    static constexpr int RFL = FF::template last_of<F...>();
    static constexpr int RIL = FF::template last_of<I...>();
    static_assert(RIL == RF0, "inverse plan must be the reversed forward plan");

    __device__ static void body(const KP &k) {
        __shared__ cf lds[BATCH * Lds<L>::RS];
        const int tid = threadIdx.x;
        const int r0 = blockIdx.x * BATCH;
        const PssPipeline &p = k.p;
        const bool re_in = p.data_in_fft != 0;
        // source -> LDS
        for (int it = tid; it < BATCH * L / 4; it += T) {
            const int b = it / (L / 4);
            const int n0 = (it - b * (L / 4)) * 4;
            float re[4], im[4];
            if (r0 + b < p.nchan) source4(k, r0 + b, n0, 4, re, im, re_in);
            else { for (int i = 0; i < 4; ++i) { re[i] = 0.f; im[i] = 0.f; } }
#pragma unroll
            for (int i = 0; i < 4; ++i) lds[Lds<L>::at(b, n0 + i)] = make_float2(re[i], im[i]);
        }
        __syncthreads();
        cf v[E];
        FF::template load<RF0>(v, lds, tid);
        __syncthreads();
        FF::template run<false, 1, F...>(v, lds, tid);
        // ramp on natural-order spectrum (last forward stage mapping)
#pragma unroll
        for (int i = 0; i < E; ++i) {
            int b, pos;
            FF::template where<RFL>(i, tid, b, pos);
            const int rr = min(r0 + b, p.nchan - 1);
            v[i] = apply_ramp(k, rr, pos, v[i]);
        }
        FF::template run<true, 1, I...>(v, lds, tid);
        FF::template store<RIL>(v, lds, tid);
        __syncthreads();
        for (int it = tid; it < BATCH * L / 4; it += T) {
            const int b = it / (L / 4);
            const int n0 = (it - b * (L / 4)) * 4;
            if (r0 + b >= p.nchan) continue;
            float pre[4], msk[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                cf z = lds[Lds<L>::at(b, n0 + i)];
                pre[i] = z.x * k.invN;
                msk[i] = z.y * k.invN;
            }
            epilogue4(k, r0 + b, n0, 4, pre, msk, !re_in);
        }
    }
};

template <typename SP, int T>
__global__ __launch_bounds__(T) void k_single(KP k) { SP::body(k); }

// ---------------------------------------------------------------------------
// path 2: four-step, N = N1 * N2, sample n = N2*n1 + n2, bin k = k1 + N1*k2.
//   A: per (row, block of B columns n2): source, FFT over n1, * W_N^{n2 k1},
//      store Y[row][k1][n2]                                  (work, complex)
//   B: per (row, BR rows k1): FFT over n2 -> ramp(k) -> inverse FFT over k2
//   C: per (row, block of B columns n2): * W_N^{-k1 n2}, inverse FFT over k1,
//      epilogue (null / out / noise), store data[row][N2*n1 + n2]
// ---------------------------------------------------------------------------
template <int N1, int B, int T, typename FWD, typename INV>
struct Cols;

template <int N1, int B, int T, int... F, int... I>
struct Cols<N1, B, T, RList<F...>, RList<I...>> {
    using FF = Fft<N1, B, T>;
    static constexpr int E = FF::E;
    static constexpr int RF0 = FF::template first<F...>();
    static constexpr int RFL = FF::template last_of<F...>();
    static constexpr int RI0 = FF::template first<I...>();
    static constexpr int RIL = FF::template last_of<I...>();

    __device__ static void passA(const KP &k) {
        __shared__ cf lds[B * Lds<N1>::RS];
        const int tid = threadIdx.x;
        const int r = blockIdx.y;
        const int64_t n20 = (int64_t)blockIdx.x * B;
        const int64_t N2 = k.N2;
        const bool re_in = k.p.data_in_fft != 0;
        for (int it = tid; it < N1 * B / 4; it += T) {
            const int n1 = it / (B / 4);
            const int b4 = (it - n1 * (B / 4)) * 4;
            float re[4], im[4];
            source4(k, r, n1 * N2 + n20 + b4, 4, re, im, re_in);
#pragma unroll
            for (int i = 0; i < 4; ++i) lds[Lds<N1>::at(b4 + i, n1)] = make_float2(re[i], im[i]);
        }
        __syncthreads();
        cf v[E];
        FF::template load<RF0>(v, lds, tid);
        __syncthreads();
        FF::template run<false, 1, F...>(v, lds, tid);
        const float invN = k.invN;
#pragma unroll
        for (int i = 0; i < E; ++i) {
            int b, k1;
            FF::template where<RFL>(i, tid, b, k1);
            int64_t m = (n20 + b) * (int64_t)k1;          // < N
            float rev = (float)m * invN;
            if (rev >= 0.5f) rev -= 1.0f;
            v[i] = cmul(v[i], expi_rev(-rev));
        }
        FF::template store<RFL>(v, lds, tid);
        __syncthreads();
        cf *Y = reinterpret_cast<cf *>(k.p.work) + (int64_t)r * k.N;
        for (int it = tid; it < N1 * B / 4; it += T) {
            const int k1 = it / (B / 4);
            const int b4 = (it - k1 * (B / 4)) * 4;
            cf a0 = lds[Lds<N1>::at(b4 + 0, k1)], a1 = lds[Lds<N1>::at(b4 + 1, k1)];
            cf a2 = lds[Lds<N1>::at(b4 + 2, k1)], a3 = lds[Lds<N1>::at(b4 + 3, k1)];
            float4 *dst = reinterpret_cast<float4 *>(Y + (int64_t)k1 * N2 + n20 + b4);
            dst[0] = make_float4(a0.x, a0.y, a1.x, a1.y);
            dst[1] = make_float4(a2.x, a2.y, a3.x, a3.y);
        }
    }

    __device__ static void passC(const KP &k) {
        __shared__ cf lds[B * Lds<N1>::RS];
        const int tid = threadIdx.x;
        const int r = blockIdx.y;
        const int64_t n20 = (int64_t)blockIdx.x * B;
        const int64_t N2 = k.N2;
        const float invN = k.invN;
        const cf *Y = reinterpret_cast<const cf *>(k.p.work) + (int64_t)r * k.N;
        for (int it = tid; it < N1 * B / 4; it += T) {
            const int k1 = it / (B / 4);
            const int b4 = (it - k1 * (B / 4)) * 4;
            const float4 *src = reinterpret_cast<const float4 *>(Y + (int64_t)k1 * N2 + n20 + b4);
            float4 lo = src[0], hi = src[1];
            cf a[4] = {make_float2(lo.x, lo.y), make_float2(lo.z, lo.w),
                       make_float2(hi.x, hi.y), make_float2(hi.z, hi.w)};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int64_t m = (n20 + b4 + i) * (int64_t)k1;
                float rev = (float)m * invN;
                if (rev >= 0.5f) rev -= 1.0f;
                lds[Lds<N1>::at(b4 + i, k1)] = cmul(a[i], expi_rev(rev));
            }
        }
        __syncthreads();
        cf v[E];
        FF::template load<RI0>(v, lds, tid);
        __syncthreads();
        FF::template run<true, 1, I...>(v, lds, tid);
        FF::template store<RIL>(v, lds, tid);
        __syncthreads();
        const bool re_in = k.p.data_in_fft != 0;
        for (int it = tid; it < N1 * B / 4; it += T) {
            const int n1 = it / (B / 4);
            const int b4 = (it - n1 * (B / 4)) * 4;
            float pre[4], msk[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                cf z = lds[Lds<N1>::at(b4 + i, n1)];
                pre[i] = z.x * invN;
                msk[i] = z.y * invN;
            }
            epilogue4(k, r, n1 * N2 + n20 + b4, 4, pre, msk, !re_in);
        }
    }
};

template <typename C, int T>
__global__ __launch_bounds__(T) void k_colA(KP k) { C::passA(k); }
template <typename C, int T>
__global__ __launch_bounds__(T) void k_colC(KP k) { C::passC(k); }

template <int N2, int BR, int T, typename FWD, typename INV, bool FWD_ONLY = false>
struct Rows;

template <int N2, int BR, int T, int... F, int... I, bool FWD_ONLY>
struct Rows<N2, BR, T, RList<F...>, RList<I...>, FWD_ONLY> {
    using FF = Fft<N2, BR, T>;
    static constexpr int E = FF::E;
    static constexpr int RF0 = FF::template first<F...>();
    static constexpr int RFL = FF::template last_of<F...>();
    static constexpr int RIL = FF::template last_of<I...>();
    static_assert(RIL == RF0, "inverse plan must be the reversed forward plan");

    __device__ static void pass(const KP &k) {
        __shared__ cf lds[BR * Lds<N2>::RS];
        const int tid = threadIdx.x;
        const int r = blockIdx.y;
        const int64_t k10 = (int64_t)blockIdx.x * BR;
        cf *Y = reinterpret_cast<cf *>(k.p.work) + (int64_t)r * k.N + k10 * N2;
        cf v[E];
        constexpr int LR = N2 / RF0;
#pragma unroll
        for (int ib = 0; ib < E / RF0; ++ib) {
            const int j = tid + ib * T, b = j / LR, jj = j - b * LR;
#pragma unroll
            for (int q = 0; q < RF0; ++q) v[ib * RF0 + q] = Y[(int64_t)b * N2 + jj + q * LR];
        }
        FF::template run<false, 1, F...>(v, lds, tid);
        if constexpr (FWD_ONLY) {
            // spectrum in natural k2 order per row k1 (mask spectrum for pair mode)
#pragma unroll
            for (int i = 0; i < E; ++i) {
                int b, k2;
                FF::template where<RFL>(i, tid, b, k2);
                Y[(int64_t)b * N2 + k2] = v[i];
            }
            return;
        }
        const int64_t N1 = k.N1;
#pragma unroll
        for (int i = 0; i < E; ++i) {
            int b, k2;
            FF::template where<RFL>(i, tid, b, k2);
            v[i] = apply_ramp(k, r, k10 + b + N1 * (int64_t)k2, v[i]);
        }
        __syncthreads();   // LDS reuse by the inverse's first exchange
        FF::template run<true, 1, I...>(v, lds, tid);
#pragma unroll
        for (int ib = 0; ib < E / RF0; ++ib) {
            const int j = tid + ib * T, b = j / LR, jj = j - b * LR;
#pragma unroll
            for (int q = 0; q < RF0; ++q) Y[(int64_t)b * N2 + jj + q * LR] = v[ib * RF0 + q];
        }
    }
};

template <typename R, int T>
__global__ __launch_bounds__(T) void k_row(KP k) { R::pass(k); }

// ---------------------------------------------------------------------------
// path 2b: four-step in PAIR mode.  Two channels a = 2p, b = 2p+1 share one
// complex row z = d_a + i d_b (half the spill bytes and half the column FFTs).
// The row pass separates their spectra with the Hermitian pairing
//   D_a(k) = (Z(k) + conj Z(N-k)) / 2,   D_b(k) = (Z(k) - conj Z(N-k)) / 2i,
// bin N-k of row k1 living in row N1-k1 (column N2-1-k2; row 0 and N1/2 pair
// with themselves), applies each channel's ramp and recombines
// W = D_a R_a + i D_b R_b before the inverse.  A delayed-null mask (same row
// for every channel) is transformed once per run (Mspec) and turned into the
// pair V = M R'_a + i M R'_b by the row pass, spilled, and inverted by pass C
// next to the data.
// ---------------------------------------------------------------------------
// Ramps in the row pass.  A thread's last-stage (radix RFL) group holds bins
// kb = kb0 + q N/RFL (q < RFL, kb0 < N/RFL); the reference's phase
// kb' s / N (kb' = kb - N above N/2) is, in 64-bit fixed point,
//   kb0 w + q (N/RFL) w - [2q >= RFL] N w   (mod 2^64, w = ramp word),
// so per bin only a 64-bit add of a uniform (scalar) offset is needed --
// bit-identical to multiplying kb' w directly.
template <int RFL>
__device__ __forceinline__ cf ramp_q(uint64_t p0, uint64_t step, uint64_t nw, int q) {
    uint64_t ph = p0 + (uint64_t)q * step;
    if (2 * q >= RFL) ph -= nw;                 // q is a compile-time constant here
    return expi_rev(-fix_to_rev(ph));
}

// Pair form of the ramps.  With R_a = e^{-2 pi i k' w_a / 2^64} and R_b the
// two channels' ramps, the recombined bin W = D_a R_a + i D_b R_b of the pair
// row (D_a = (Z + conj Zm)/2, D_b = (Z - conj Zm)/2i) is
//     W = E (Z cos d - i conj(Zm) sin d),   E = e^{-i (alpha + beta)/2},
//                                           d = (alpha - beta)/2,
// because (R_a + R_b)/2 = E cos d and (R_a - R_b)/2 = -i E sin d.  E and
// D = e^{-i d} come from the half words h = w >> 1 (h_a + h_b and h_a - h_b):
// any h with 2h = w mod 2^64 gives the same W (a dropped top bit flips E and
// D together by (-1)^k'), so no extra host data is needed.  Per bin that is
// two complex products for E and D (base(kb0) x table[q], as before) plus
// four products and one complex product for W: 16 VALU instead of 22.
// Per-pair factors: bin kb0 + q N/RFL has phase offset q (N/RFL) h - [2q >=
// RFL] N h relative to kb0; tabulated once per run in double precision,
// tab[pair][q] = {E factor, D factor}.
template <int RFL>
__global__ void k_pair_tab(const uint64_t *ramp, int64_t N, int nchan, int poff, int npairs, cf *tab) {
    const int pr = blockIdx.x, q = threadIdx.x;
    if (pr >= npairs || q >= RFL) return;
    const int ra = max(2 * pr - poff, 0), rb = min(2 * pr + 1 - poff, nchan - 1);
    const uint64_t ha = (uint64_t)ramp[ra] >> 1, hb = (uint64_t)ramp[rb] >> 1;
    const uint64_t h2[2] = {ha + hb, ha - hb};
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        uint64_t ph = (uint64_t)q * ((uint64_t)(N / RFL) * h2[e]);
        if (2 * q >= RFL) ph -= (uint64_t)N * h2[e];
        const double rev = (double)(int64_t)ph * 5.421010862427522e-20;   // 2^-64
        double sn, cs;
        sincospi(2.0 * rev, &sn, &cs);
        tab[((int64_t)pr * RFL + q) * 2 + e] = make_float2((float)cs, (float)(-sn));
    }
}

template <int N2, int T, typename FWD, typename INV>
struct PairRows;

template <int N2, int T, int... F, int... I>
struct PairRows<N2, T, RList<F...>, RList<I...>> {
    // row pitch N2 + 16 (a multiple of 16 complex: the byte-address XOR
    // exchanges, Fft::XB; the rows' bank offset is irrelevant here -- every
    // wave works on one row per instruction)
    using FF = Fft<N2, 2, T, false, 16>;
    using LD = typename FF::LD;
    static constexpr int E = FF::E;
    static constexpr int RF0 = FF::template first<F...>();
    static constexpr int RFL = FF::template last_of<F...>();
    static constexpr int RIL = FF::template last_of<I...>();
    static_assert(RIL == RF0, "inverse plan must be the reversed forward plan");
    static constexpr int LR = N2 / RF0;
    static constexpr int LRL = N2 / RFL;
    // minimum waves per SIMD the kernel is compiled for (VGPR budget 512 /
    // waves): two workgroups per CU when two rows fit twice in LDS
    static constexpr int kMinWaves = (T <= 512) ? 2 * T / 256 : 4;
    // byte offset of (row, n2) in a pair spill, and the offset step of the
    // q-th first-stage input (n2 + q LR)
    static constexpr uint32_t kQS = 8u * (uint32_t)LR;
    __device__ static __forceinline__ uint32_t spill_off(uint32_t RP, int row, int n2) {
        return ((uint32_t)row * RP + (uint32_t)n2) * 8u;
    }

    // MASK = false: data pair of channels (2pr - poff, 2pr + 1 - poff).
    // MASK = true : node pair (2pr, 2pr + 1) of the mask table build -- the
    //               once-per-run mask spectrum times each node's ramp.
    // HT: a per-bin transfer function H (PssPipeline.htab: the baseband
    // coherent dispersion, ism.py:76-98) instead of the delay ramps -- one H
    // for every channel, so the packed pair's bins are simply H_ext(k) Z(k)
    // (H_ext(N - k) = conj H(k); DC and Nyquist x Re H, the irfft rule).
    template <bool MASK, bool TAIL = false, bool HT = false>
    __device__ static void pass(const KP &k) {
        __shared__ __align__(128) cf lds[2 * LD::RS];
        __shared__ cf tw16[kTw16Size];
        const int tid = threadIdx.x;
        tw16_fill(tw16, tid, T);     // first read after the first stage's barrier
        const int pr = blockIdx.x;                 // channel pair
        const int j = blockIdx.y;                  // row pair {j, N1-j}; {0, N1/2}
        const int N1 = (int)k.N1;
        const int rowA = j, rowB = (j == 0) ? N1 / 2 : N1 - j;
        const int off = MASK ? 0 : k.poff;
        const int ra = max(2 * pr - off, 0), rb = min(2 * pr + 1 - off, k.p.nchan - 1);
        const bool data = !MASK;
        const bool mask = MASK;
        const uint64_t rwa = HT ? 0ull : (uint64_t)k.p.ramp[ra], rwb = HT ? 0ull : (uint64_t)k.p.ramp[rb];
        // uniform 64-bit phase offsets of bin kb0 + q N/RFL relative to kb0 (SALU)
        const uint64_t sta = (uint64_t)(k.N / RFL) * rwa, stb = (uint64_t)(k.N / RFL) * rwb;
        const uint64_t nwa = (uint64_t)k.N * rwa, nwb = (uint64_t)k.N * rwb;
        cf v[E];
        const uint32_t pbytes = (uint32_t)(pstride(k) * 8);
        const uint32_t RP = (uint32_t)rpitch(k);
        if (data) {
            const Buf Y(k.Yd + (int64_t)pr * pstride(k), pbytes);
#pragma unroll
            for (int ib = 0; ib < E / RF0; ++ib) {
                const int jj0 = tid + ib * T, b = jj0 / LR, jj = jj0 - b * LR;
                const uint32_t off = spill_off(RP, b ? rowB : rowA, jj);
#pragma unroll
                for (int q = 0; q < RF0; ++q) v[ib * RF0 + q] = Y.ld2(off, q * kQS);
            }
            FF::template run_tw<false, 1, F...>(v, lds, tid, tw16);
            if constexpr (HT) {
                // bin kb0 + q N/RFL of butterfly ib (no mirror bins needed)
                const cf *H = reinterpret_cast<const cf *>(k.p.htab);
#pragma unroll
                for (int ib = 0; ib < E / RFL; ++ib) {
                    const int jg = tid + ib * T, b = jg / LRL, jj = jg - b * LRL;
                    const int64_t kb0 = (b ? rowB : rowA) + (int64_t)N1 * jj;
#pragma unroll
                    for (int q = 0; q < RFL; ++q) {
                        const int64_t kb = kb0 + (int64_t)q * (k.N / RFL);
                        const bool upper = 2 * kb > k.N;
                        const cf h = H[upper ? k.N - kb : kb];
                        cf &z = v[ib * RFL + q];
                        if (kb == 0 || 2 * kb == k.N) z = make_float2(z.x * h.x, z.y * h.x);
                        else z = cmul(z, make_float2(h.x, upper ? -h.y : h.y));
                    }
                }
            } else {
            FF::template store<RFL>(v, lds, tid);
            __syncthreads();
            // pair ramp factors (k_pair_tab): {E, D} per q, wave-uniform
            const cf *ptab = k.rtab + (int64_t)pr * (2 * RFL);
            const uint64_t hsum = (rwa >> 1) + (rwb >> 1), hdif = (rwa >> 1) - (rwb >> 1);
            // RFL = 16 (the C3 4096-point rows): the bins of a butterfly as one
            // straight-line body under a scalar branch (the form below measured
            // neutral at C3 and 0.8 ms slower on C5's 8192-point rows, RFL = 8,
            // profiles/r03/s6: those keep the per-bin form)
            if constexpr (RFL == 16) {
#pragma unroll
            for (int ib = 0; ib < E / RFL; ++ib) {
                const int jg = tid + ib * T;
                // row side b is wave-uniform when LRL is a multiple of the
                // wave: say so, so the mirror-read choice below is a scalar branch
                const int b = (LRL % 64 == 0) ? __builtin_amdgcn_readfirstlane(jg / LRL) : jg / LRL;
                const int jj = jg - b * LRL;
                const int row = b ? rowB : rowA;
                const int64_t kb0 = row + (int64_t)N1 * jj;
                const cf bE = expi_rev(-fix_to_rev((uint64_t)kb0 * hsum));
                const cf bD = expi_rev(-fix_to_rev((uint64_t)kb0 * hdif));
                const bool dc = (kb0 == 0);                      // one lane of one wave per launch
                // bin q of this butterfly from Z = v[i] and its mirror Zm:
                // W = D_a R_a + i D_b R_b; DC (q = 0) and Nyquist (q = RFL/2)
                // of kb0 = 0 by select (no per-bin branch: the body stays
                // straight-line, so the mirror reads of several bins are in
                // flight together)
                auto bin = [&](int q, cf Zm) {
                    const int i = ib * RFL + q;
                    const cf Z = v[i];
                    // 2 D_a and 2 D_b (DC / Nyquist and the tail extension)
                    const cf Sa = make_float2(Z.x + Zm.x, Z.y - Zm.y);
                    const cf Sb = make_float2(Z.y + Zm.y, Zm.x - Z.x);
                    cf W;
                    {
                        const cf Ef = cmul(bE, ptab[2 * q]), Df = cmul(bD, ptab[2 * q + 1]);
                        if constexpr (TAIL) {
                            // per-channel transfer functions: R_a = E D, R_b = E conj(D)
                            const cf w = bin_phasor(kb0 + (int64_t)q * (k.N / RFL), k.N);
                            const cf ra_ = cmul(make_float2(0.5f * Ef.x, 0.5f * Ef.y), cmul(Df, tail_factor(k.p.tail_a[ra], w)));
                            const cf rb_ = cmul(make_float2(0.5f * Ef.x, 0.5f * Ef.y), cmul_conj(tail_factor(k.p.tail_a[rb], w), Df));
                            const cf A = cmul(Sa, ra_);
                            const cf Bv = cmul(Sb, rb_);
                            W = make_float2(A.x - Bv.y, A.y + Bv.x);
                        } else {
                            // W = E (Z cos d - i conj(Zm) sin d), D = cos d - i sin d
                            const float c = Df.x, s = -Df.y;
                            const cf in = make_float2(fmaf(Z.x, c, -(Zm.y * s)), fmaf(Z.y, c, -(Zm.x * s)));
                            W = cmul(Ef, in);
                        }
                        if (2 * q == RFL) {                         // Nyquist bin (compile-time q)
                            float fa = k.p.nyq_re[ra], fb = k.p.nyq_re[rb];
                            if constexpr (TAIL) {                   // H(N/2) = (1-a)/(1+a)
                                const float ta = k.p.tail_a[ra], tb = k.p.tail_a[rb];
                                fa *= (1.0f - ta) / (1.0f + ta);
                                fb *= (1.0f - tb) / (1.0f + tb);
                            }
                            const cf Wn = make_float2((0.5f * Sa.x) * fa, (0.5f * Sb.x) * fb);
                            W = dc ? Wn : W;
                        } else if (q == 0) {                        // DC (H = 1)
                            const cf Da = make_float2(0.5f * Sa.x, 0.5f * Sa.y), Db = make_float2(0.5f * Sb.x, 0.5f * Sb.y);
                            const cf Wd = make_float2(Da.x - Db.y, Da.y + Db.x);
                            W = dc ? Wd : W;
                        }
                    }
                    v[i] = W;
                };
                // mirror bins k2m = N2 - 1 - k2 = P0 - q LRL (all but row 0 of
                // the {0, N1/2} pair, whose bin 0 pairs with itself): with
                // LRL % 256 == 0 the swizzle XOR is the same for every q, so
                // the reads are one byte base minus immediate offsets.  The
                // choice is one scalar branch around the whole bin loop.
                constexpr bool kMirXB = FF::XB && (LRL % 256 == 0);
                const bool affine = !(j == 0 && row == 0);       // wave-uniform
                if (kMirXB && affine) {
                    const uint32_t mbase = lds_byte(lds) + 8u * (uint32_t)LD::at(j == 0 ? b : 1 - b, N2 - 1 - jj);
#pragma unroll
                    for (int q = 0; q < RFL; ++q) bin(q, lds_ld(mbase - 8u * (uint32_t)(q * LRL)));
                } else {
#pragma unroll
                    for (int q = 0; q < RFL; ++q) {
                        const int k2 = jj + q * LRL;
                        int bm, k2m;
                        if (j == 0) { bm = b; k2m = (row == 0) ? (((N2 & (N2 - 1)) == 0) ? ((N2 - k2) & (N2 - 1)) : (k2 ? N2 - k2 : 0)) : (N2 - 1 - k2); }
                        else        { bm = 1 - b; k2m = N2 - 1 - k2; }
                        bin(q, lds[LD::at(bm, k2m)]);
                    }
                }
            }
            } else {
#pragma unroll
            for (int ib = 0; ib < E / RFL; ++ib) {
                const int jg = tid + ib * T, b = jg / LRL, jj = jg - b * LRL;
                const int row = b ? rowB : rowA;
                const int64_t kb0 = row + (int64_t)N1 * jj;
                const cf bE = expi_rev(-fix_to_rev((uint64_t)kb0 * hsum));
                const cf bD = expi_rev(-fix_to_rev((uint64_t)kb0 * hdif));
                // mirror bins k2m = N2 - 1 - k2 = P0 - q LRL (all but row 0 of
                // the {0, N1/2} pair, whose bin 0 pairs with itself): with
                // LRL % 256 == 0 the swizzle XOR is the same for every q, so
                // the reads are one byte base minus immediate offsets
                constexpr bool kMirXB = FF::XB && (LRL % 256 == 0);
                const bool affine = !(j == 0 && row == 0);       // wave-uniform
                uint32_t mbase = 0;
                if constexpr (kMirXB) mbase = lds_byte(lds) + 8u * (uint32_t)LD::at(j == 0 ? b : 1 - b, N2 - 1 - jj);
#pragma unroll
                for (int q = 0; q < RFL; ++q) {
                    const int i = ib * RFL + q, k2 = jj + q * LRL;
                    cf Zm;
                    if (kMirXB && affine) {
                        Zm = lds_ld(mbase - 8u * (uint32_t)(q * LRL));
                    } else {
                        int bm, k2m;
                        if (j == 0) { bm = b; k2m = (row == 0) ? (((N2 & (N2 - 1)) == 0) ? ((N2 - k2) & (N2 - 1)) : (k2 ? N2 - k2 : 0)) : (N2 - 1 - k2); }
                        else        { bm = 1 - b; k2m = N2 - 1 - k2; }
                        Zm = lds[LD::at(bm, k2m)];
                    }
                    const cf Z = v[i];
                    // 2 D_a and 2 D_b (DC / Nyquist and the tail extension)
                    const cf Sa = make_float2(Z.x + Zm.x, Z.y - Zm.y);
                    const cf Sb = make_float2(Z.y + Zm.y, Zm.x - Z.x);
                    if (kb0 == 0 && 2 * q == RFL) {                 // Nyquist bin
                        float fa = k.p.nyq_re[ra], fb = k.p.nyq_re[rb];
                        if constexpr (TAIL) {                       // H(N/2) = (1-a)/(1+a)
                            const float ta = k.p.tail_a[ra], tb = k.p.tail_a[rb];
                            fa *= (1.0f - ta) / (1.0f + ta);
                            fb *= (1.0f - tb) / (1.0f + tb);
                        }
                        v[i] = make_float2((0.5f * Sa.x) * fa, (0.5f * Sb.x) * fb);
                    } else if (kb0 == 0 && q == 0) {                // DC (H = 1)
                        const cf Da = make_float2(0.5f * Sa.x, 0.5f * Sa.y), Db = make_float2(0.5f * Sb.x, 0.5f * Sb.y);
                        v[i] = make_float2(Da.x - Db.y, Da.y + Db.x);
                    } else {
                        const cf Ef = cmul(bE, ptab[2 * q]), Df = cmul(bD, ptab[2 * q + 1]);
                        if constexpr (TAIL) {
                            // per-channel transfer functions: R_a = E D, R_b = E conj(D)
                            const cf w = bin_phasor(kb0 + (int64_t)q * (k.N / RFL), k.N);
                            const cf ra_ = cmul(make_float2(0.5f * Ef.x, 0.5f * Ef.y), cmul(Df, tail_factor(k.p.tail_a[ra], w)));
                            const cf rb_ = cmul(make_float2(0.5f * Ef.x, 0.5f * Ef.y), cmul_conj(tail_factor(k.p.tail_a[rb], w), Df));
                            const cf A = cmul(Sa, ra_);
                            const cf Bv = cmul(Sb, rb_);
                            v[i] = make_float2(A.x - Bv.y, A.y + Bv.x);
                        } else {
                            // W = E (Z cos d - i conj(Zm) sin d), D = cos d - i sin d
                            const float c = Df.x, s = -Df.y;
                            const cf in = make_float2(fmaf(Z.x, c, -(Zm.y * s)), fmaf(Z.y, c, -(Zm.x * s)));
                            v[i] = cmul(Ef, in);
                        }
                    }
                }
            }
            }
            }   // (HT)
            __syncthreads();
            FF::template run_tw<true, 1, I...>(v, lds, tid, tw16);
#pragma unroll
            for (int ib = 0; ib < E / RF0; ++ib) {
                const int jj0 = tid + ib * T, b = jj0 / LR, jj = jj0 - b * LR;
                const uint32_t off = spill_off(RP, b ? rowB : rowA, jj);
#pragma unroll
                for (int q = 0; q < RF0; ++q) Y.st2(v[ib * RF0 + q], off, q * kQS);
            }
        }
        if (mask) {
            const Buf V(k.Ym + (int64_t)pr * pstride(k), pbytes);
            const Buf Ms(k.Mspec, (uint32_t)(k.N * 8));      // [N1][N2], no spill pad
#pragma unroll
            for (int ib = 0; ib < E / RFL; ++ib) {
                const int jg = tid + ib * T, b = jg / LRL, jj = jg - b * LRL;
                const int row = b ? rowB : rowA;
                const int64_t kb0 = row + (int64_t)N1 * jj;
                const uint64_t p0a = (uint64_t)kb0 * rwa, p0b = (uint64_t)kb0 * rwb;
                const uint32_t moff = (uint32_t)(row * N2 + jj) * 8u;
#pragma unroll
                for (int q = 0; q < RFL; ++q) {
                    const int i = ib * RFL + q;
                    const cf M = Ms.ld2(moff, q * LRL * 8);
                    if (kb0 == 0 && 2 * q == RFL) {                 // Nyquist bin
                        v[i] = make_float2(M.x * k.p.nyq_im[ra], M.x * k.p.nyq_im[rb]);
                    } else if (kb0 == 0 && q == 0) {                // DC: M (1 + i)
                        v[i] = make_float2(M.x - M.y, M.y + M.x);
                    } else {                                        // M (R_a + i R_b)
                        const cf Ra = ramp_q<RFL>(p0a, sta, nwa, q), Rb = ramp_q<RFL>(p0b, stb, nwb, q);
                        v[i] = cmul(M, make_float2(Ra.x - Rb.y, Ra.y + Rb.x));
                    }
                }
            }
            __syncthreads();
            FF::template run_tw<true, 1, I...>(v, lds, tid, tw16);
#pragma unroll
            for (int ib = 0; ib < E / RF0; ++ib) {
                const int jj0 = tid + ib * T, b = jj0 / LR, jj = jj0 - b * LR;
                const uint32_t off = spill_off(RP, b ? rowB : rowA, jj);
#pragma unroll
                for (int q = 0; q < RF0; ++q) V.st2(v[ib * RF0 + q], off, q * kQS);
            }
        }
    }
};

template <typename R, int T, bool TAIL = false, bool HT = false>
__global__ __launch_bounds__(T, R::kMinWaves) void k_pair_row(KP k) { R::template pass<false, TAIL, HT>(k); }
template <typename R, int T>
__global__ __launch_bounds__(T) void k_node_row(KP k) { R::template pass<true>(k); }

// Row pass of a data pair with the two rows of a row pair in registers and
// ONE row in LDS (the 8192-point rows of C5's 2048 x 8192
// split): PairRows holds both rows in LDS (2 x 65.7 KB, one workgroup per
// CU, so every barrier stalls the CU); here each exchange moves one row
// through a 65.7-KB buffer and two workgroups share a CU.  Same stages and
// ramp arithmetic as PairRows::pass<false> (no tail extension).  After the
// forward transforms a thread holds row A's bins k2 = jj + q LRL and row
// B's at the mirrors N2-1-k2 (row B's thread relabelling below); it forms
// W_A(k2) and W_B(N2-1-k2) from the same pair of registers.  Row pair {0,
// N1/2} (each row its own mirror, DC and Nyquist in row 0) takes the
// per-row form through LDS.
template <int N2, int T, typename FWD, typename INV>
struct PairRowsSeq;

// a value the compiler cannot see through (no CSE across uses)
__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

template <int N2, int T, int... F, int... I>
struct PairRowsSeq<N2, T, RList<F...>, RList<I...>> {
    using FF = Fft<N2, 1, T, false, 16>;
    using LD = typename FF::LD;
    using PRW = PairRows<N2, T, RList<F...>, RList<I...>>;   // spill addressing
    static constexpr int E = FF::E;                           // values per thread of ONE row
    static constexpr int RF0 = FF::template first<F...>();
    static constexpr int RFL = FF::template last_of<F...>();
    static constexpr int LR = N2 / RF0;
    static constexpr int LRL = N2 / RFL;
    static_assert(FF::template last_of<I...>() == RF0 && FF::template first<I...>() == RFL,
                  "inverse plan must be the reversed forward plan");
    static_assert(E / RF0 * T <= LR && E / RFL * T <= LRL, "one row per thread mapping");

    // W = E (Z cos d - i conj(Zm) sin d) of bin kb0 + q N/RFL (PairRows::pass)
    __device__ static __forceinline__ cf ramp(cf Z, cf Zm, cf bE, cf bD, const cf *ptab, int q) {
        const cf Ef = cmul(bE, ptab[2 * q]), Df = cmul(bD, ptab[2 * q + 1]);
        const float c = Df.x, s = -Df.y;
        return cmul(Ef, make_float2(fmaf(Z.x, c, -(Zm.y * s)), fmaf(Z.y, c, -(Zm.x * s))));
    }

    // SELF: row pair {0, N1/2} (its own launch: a branch between the two
    // forms makes the compiler spill both rows at the branch)
    template <bool SELF>
    __device__ static void pass(const KP &k) {
        __shared__ __align__(128) cf lds[LD::RS];
        __shared__ cf tw16[kTw16Size];
        const int tid = threadIdx.x;
        tw16_fill(tw16, tid, T);
        const int pr = blockIdx.x;
        const int j = SELF ? 0 : (int)blockIdx.y + 1;   // row pair {j, N1-j}; {0, N1/2}
        const int N1 = (int)k.N1;
        const int rowA = j, rowB = (j == 0) ? N1 / 2 : N1 - j;
        const int ra = max(2 * pr - k.poff, 0), rb = min(2 * pr + 1 - k.poff, k.p.nchan - 1);
        const uint64_t rwa = (uint64_t)k.p.ramp[ra], rwb = (uint64_t)k.p.ramp[rb];
        const uint64_t hsum = (rwa >> 1) + (rwb >> 1), hdif = (rwa >> 1) - (rwb >> 1);
        const cf *ptab = k.rtab + (int64_t)pr * (2 * RFL);
        const uint32_t RP = (uint32_t)rpitch(k);
        const Buf Y(k.Yd + (int64_t)pr * pstride(k), (uint32_t)(pstride(k) * 8));
        cf va[E], vb[E];
        // one row's registers live across the other's transform, not two
        // rows' loads in flight (the 128-VGPR budget of 4 waves per SIMD)
        auto load = [&](cf (&v)[E], int row, int b, int t) __attribute__((always_inline)) {
#pragma unroll
            for (int ib = 0; ib < E / RF0; ++ib) {
                const uint32_t o = PRW::spill_off(RP, row, t + ib * T);
#pragma unroll
                for (int q = 0; q < RF0; ++q) v[ib * RF0 + q] = Y.ld2(o, q * PRW::kQS);
            }
        };
        // Row B runs as thread tb = T-1-tid (a relabelling of the threads:
        // every stage and both spill accesses use tb).  With LRL = (E/RFL) T
        // its last forward stage leaves, in register E-1-i, row B's bin
        // N2-1-k2 -- the mirror of row A's bin k2 in register i -- so the
        // ramp pairs registers without an LDS exchange, and W_B is already
        // in thread tb's inverse input mapping.
        const int tb = SELF ? tid : T - 1 - tid;
        // (each transform ends with a barrier after its last LDS read, so
        // the next one may scatter at once)
        // opaque(...) per transform: the four transforms have identical
        // LDS address arithmetic, and without it the compiler keeps one
        // set of addresses live across the kernel (spilled) instead of
        // recomputing them
        load(va, rowA, 0, tid);
        FF::template run_tw<false, 1, F...>(va, lds, opaque(tid), tw16);
        load(vb, rowB, 1, tb);
        FF::template run_tw<false, 1, F...>(vb, lds, opaque(tb), tw16);
        if constexpr (!SELF) {
            static_assert(E / RFL * T == LRL, "mirror registers need LRL = (E/RFL) T");
#pragma unroll
            for (int ib = 0; ib < E / RFL; ++ib) {
                const int jj = tid + ib * T, jm = LRL - 1 - jj;
                const int64_t ka = rowA + (int64_t)N1 * jj, kbm = rowB + (int64_t)N1 * jm;
                const cf aE = expi_rev(-fix_to_rev((uint64_t)ka * hsum));
                const cf aD = expi_rev(-fix_to_rev((uint64_t)ka * hdif));
                const cf bE = expi_rev(-fix_to_rev((uint64_t)kbm * hsum));
                const cf bD = expi_rev(-fix_to_rev((uint64_t)kbm * hdif));
#pragma unroll
                for (int q = 0; q < RFL; ++q) {
                    const int i = ib * RFL + q;
                    const cf Za = va[i], Zb = vb[E - 1 - i];      // A at k2, B at N2-1-k2
                    va[i] = ramp(Za, Zb, aE, aD, ptab, q);
                    vb[E - 1 - i] = ramp(Zb, Za, bE, bD, ptab, RFL - 1 - q);
                }
            }
        } else {
            // rows 0 and N1/2: each its own mirror (row 0: bin 0 with itself)
            auto self = [&](cf (&v)[E], int row) __attribute__((always_inline)) {
                FF::template store<RFL>(v, lds, opaque(tid));
                __syncthreads();
#pragma unroll
                for (int ib = 0; ib < E / RFL; ++ib) {
                    const int jj = tid + ib * T;
                    const int64_t kb0 = row + (int64_t)N1 * jj;
                    const cf bE = expi_rev(-fix_to_rev((uint64_t)kb0 * hsum));
                    const cf bD = expi_rev(-fix_to_rev((uint64_t)kb0 * hdif));
#pragma unroll
                    for (int q = 0; q < RFL; ++q) {
                        const int i = ib * RFL + q, k2 = jj + q * LRL;
                        const int k2m = (row == 0) ? (((N2 & (N2 - 1)) == 0) ? ((N2 - k2) & (N2 - 1)) : (k2 ? N2 - k2 : 0)) : (N2 - 1 - k2);
                        const cf Z = v[i], Zm = lds[LD::at(0, k2m)];
                        const cf Sa = make_float2(Z.x + Zm.x, Z.y - Zm.y);
                        const cf Sb = make_float2(Z.y + Zm.y, Zm.x - Z.x);
                        if (kb0 == 0 && 2 * q == RFL) {          // Nyquist bin
                            v[i] = make_float2((0.5f * Sa.x) * k.p.nyq_re[ra], (0.5f * Sb.x) * k.p.nyq_re[rb]);
                        } else if (kb0 == 0 && q == 0) {         // DC (H = 1)
                            const cf Da = make_float2(0.5f * Sa.x, 0.5f * Sa.y), Db = make_float2(0.5f * Sb.x, 0.5f * Sb.y);
                            v[i] = make_float2(Da.x - Db.y, Da.y + Db.x);
                        } else {
                            v[i] = ramp(Z, Zm, bE, bD, ptab, q);
                        }
                    }
                }
                __syncthreads();
            };
            self(va, rowA);
            self(vb, rowB);
        }
        FF::template run_tw<true, 1, I...>(va, lds, opaque(tid), tw16);
#pragma unroll
        for (int ib = 0; ib < E / RF0; ++ib) {
            const int jj = tid + ib * T;
            const uint32_t oa = PRW::spill_off(RP, rowA, jj);
#pragma unroll
            for (int q = 0; q < RF0; ++q) Y.st2(va[ib * RF0 + q], oa, q * PRW::kQS);
        }
        FF::template run_tw<true, 1, I...>(vb, lds, opaque(tb), tw16);
#pragma unroll
        for (int ib = 0; ib < E / RF0; ++ib) {
            const int jj = tb + ib * T;
            const uint32_t ob = PRW::spill_off(RP, rowB, jj);
#pragma unroll
            for (int q = 0; q < RF0; ++q) Y.st2(vb[ib * RF0 + q], ob, q * PRW::kQS);
        }
    }
};

template <typename R, int T, bool SELF>
__global__ __launch_bounds__(T, SELF ? 1 : 4) void k_pair_row_seq(KP k) { R::template pass<SELF>(k); }


// XRS: extra row pitch of the LDS column block (Lds), chosen per kernel for
// its transposing accesses (xrs_read / xrs_write below).
template <int N1, int B, int T, typename FWD, typename INV, int XRS = 1>
struct PairCols;

template <int N1, int B, int T, int... F, int... I, int XRS>
struct PairCols<N1, B, T, RList<F...>, RList<I...>, XRS> {
    using LdsC = Lds<N1, XRS>;
    using FF = Fft<N1, B, T, false, XRS>;
    static constexpr int E = FF::E;
    // One wave per column (T = 64 B, N1/64 values per lane): the column FFTs
    // are wave-local (Fft<..., WAVE>: no workgroup barrier between stages);
    // only the transposes between sample-major items and columns need one.
    using FW = Fft<(N1 % 64 == 0 ? N1 : 64), 1, 64, true, XRS>;   // same row layout as LdsC (placeholder when N1 % 64 != 0)
    static constexpr bool kWaveCols = (T == 64 * B) && (N1 % 64 == 0) && (N1 / 64 == E);
    // pass A: four-step twiddle folded into the column FFT's last stage
    static constexpr bool kMergeTw = sizeof...(F) >= 2;
    static constexpr int RF0 = FF::template first<F...>();
    static constexpr int RFL = FF::template last_of<F...>();
    static constexpr int RI0 = FF::template first<I...>();
    static constexpr int RIL = FF::template last_of<I...>();
    static constexpr int ITEMS = N1 * B / 4 / T;
    // the unrolled fast kernels need a whole number of 4-sample items per
    // thread (N1 = 2^m); the generic ones loop (any N1, e.g. 30 = 2 * 3 * 5)
    static constexpr bool kItemsExact = ITEMS * 4 * T == N1 * B;
    // Mixed-radix columns (N1 not a power of two, one column per thread, B
    // == T): the column DFTs run in registers (RegDft: compile-time twiddles,
    // no LDS exchange), the spill is written / read one column per lane
    // (consecutive lanes = consecutive columns: coalesced rows)
    static constexpr bool kRegCols = (B == T) && ((N1 & (N1 - 1)) != 0);
    static constexpr int kFoldWaves = N1 <= 30 ? 4 : 2;      // min waves per SIMD of the fold kernels
    // passC_fold's lane-private LDS (N1 x 8 B per lane) caps its waves per
    // SIMD at (160 KB / (N1 x 8 B x B)) x B / 256
    static constexpr int kFoldWavesC = (160 * 1024 / (N1 * 8 * B)) * B / 256 < 1 ? 1
                                     : ((160 * 1024 / (N1 * 8 * B)) * B / 256 > 4 ? 4 : (160 * 1024 / (N1 * 8 * B)) * B / 256);
    static_assert(B % 4 == 0, "4-sample items");

    // A: generate channels a, b into z = d_a + i d_b; column FFTs; twiddle; spill.
    // FAST (host-selected): search-mode source with Philox chi2(1) draws, no
    // injected draws, no undelayed null -- the same values as source4.
    template <bool FAST, bool SHARED = false>
    __device__ static void passA(const KP &k) {
        __shared__ __align__(128) cf lds[B * LdsC::RS];   // (128-B aligned: the FFT's byte-address exchanges)
        __shared__ cf tw16[kTw16Size];
        const int tid = threadIdx.x;
        tw16_fill(tw16, tid, T);     // read after the generate loop's barrier
        int cbx, pr;
        xcd_block(cbx, pr);
        const int ra = 2 * pr - k.poff, rb = ra + 1;
        const bool hasa = ra >= 0, hasb = rb < k.p.nchan;
        const int64_t n20 = (int64_t)cbx * B;
        const int64_t N2 = k.N2;
        const PssPipeline &p = k.p;
        const uint32_t ca = (uint32_t)(p.chan0 + ra), cb = ca + 1u;
        const int pra = (p.prof_rows == 1) ? 0 : (int)ca - p.prof_row0, prb = (p.prof_rows == 1) ? 0 : (int)cb - p.prof_row0;
        const Rng g(p.seed, p.call_gen, P_PULSE);
        static_assert(!FAST || kItemsExact, "fast pass A: whole items per thread");
        if constexpr (FAST) {
            // The pair's two PCHIP rows are staged in LDS (host guarantees
            // nint <= kFastNint), the items are unrolled and branch-free, so
            // the table reads of an item issue together instead of one
            // exposed global-load latency per sample.
            __shared__ float4 ptab[2][kFastNint];
            const int nint = p.nint;
            const int last = p.prof_rows - 1;
            const int rowa = min(max(pra, 0), last), rowb = min(max(prb, 0), last);
            // SHARED (host-selected: prof_rows == 1, e.g. C3's GaussProfile):
            // one table row serves both channels, one lookup and evaluation
            constexpr bool shared = SHARED;
            const float4 *prof = reinterpret_cast<const float4 *>(p.prof);
            for (int i = tid; i < nint; i += T) {
                ptab[0][i] = prof[(int64_t)rowa * nint + i];
                if constexpr (!shared) ptab[1][i] = prof[(int64_t)rowb * nint + i];
            }
            __syncthreads();
            // draw_norm, or 0 for a pair's missing channel (shard / band
            // edges): the multiply the sample needs anyway zeroes it, no select
            const float dna = hasa ? p.draw_norm : 0.f, dnb = hasb ? p.draw_norm : 0.f;
            // item = 4 consecutive samples n .. n + 3 of row n1 (Philox block
            // n >> 2, at every N), phases by a unit walk
            uint32_t dlo;
            uint64_t dhi;
            phase_delta(p, dlo, dhi);
            const uint32_t M = p.knot_m;
#pragma unroll
            for (int t = 0; t < ITEMS; ++t) {
                // lanes = consecutive rows n1 (of one 4-column group where
                // N1 % 64 == 0): the transposed LDS writes below are
                // conflict-free (this loop touches no global memory, so its
                // item order is free)
                const int it = tid + t * T;
                int n1, b4;
                if constexpr (N1 % 64 == 0) {
                    n1 = it % N1;
                    b4 = (it / N1) * 4;
                } else {
                    n1 = it / (B / 4);
                    b4 = (it - n1 * (B / 4)) * 4;
                }
                const uint32_t n = (uint32_t)(n1 * (int)N2) + (uint32_t)n20 + (uint32_t)b4;   // N < 2^24
                // draws scaled by draw_norm (0 for a pair's missing channel) in the sampler
                const float4 qa = chi2_1x4(g.bits(n >> 2, ca, 0u), dna);
                const float4 qb = chi2_1x4(g.bits(n >> 2, cb, 0u), dnb);
                const float va[4] = {qa.x, qa.y, qa.z, qa.w}, vb[4] = {qb.x, qb.y, qb.z, qb.w};
                PhaseWalk w;
                w.start(p, n);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    uint32_t iv;
                    float u;
                    if (i) w.step(dlo, dhi, M);
                    w.get_full(iv, u);       // fast_source(): nint == knot_m
                    const float4 A = ptab[0][iv];
                    const float pa = fmaf(fmaf(fmaf(A.x, u, A.y), u, A.z), u, A.w);
                    float pb = pa;
                    if constexpr (!shared) {
                        const float4 Bc = ptab[1][iv];
                        pb = fmaf(fmaf(fmaf(Bc.x, u, Bc.y), u, Bc.z), u, Bc.w);
                    }
                    lds[LdsC::at(b4 + i, n1)] = make_float2(pa * va[i], pb * vb[i]);
                }
            }
        } else
        for (int it = tid; it < N1 * B / 4; it += T) {
            const int n1 = it / (B / 4);
            const int b4 = (it - n1 * (B / 4)) * 4;
            const int64_t n = n1 * N2 + n20 + b4;
            float xa[4], xb[4], dum[4];
            if (hasa) source4(k, ra, n, 4, xa, dum, true, false);
            else { xa[0] = xa[1] = xa[2] = xa[3] = 0.f; }
            if (hasb) source4(k, rb, n, 4, xb, dum, true, false);
            else { xb[0] = xb[1] = xb[2] = xb[3] = 0.f; }
#pragma unroll
            for (int i = 0; i < 4; ++i) lds[LdsC::at(b4 + i, n1)] = make_float2(xa[i], xb[i]);
        }
        __syncthreads();
        if constexpr (kRegCols) {
            cf x[N1];
#pragma unroll
            for (int n1 = 0; n1 < N1; ++n1) x[n1] = lds[LdsC::at(tid, n1)];
            reg_spill(k, x, pr, n20 + tid);
            return;
        }
        cf v[E];
        const float invN = k.invN;
        if constexpr (kWaveCols) {
            // wave w transforms column w in its own LDS row
            const int wv = tid >> 6, lane = tid & 63;
            cf *wl = lds + wv * LdsC::RS;
            FW::template load<RF0>(v, wl, lane);
            stage_sync<true>();
            if constexpr (kMergeTw) {
                // Last stage (radix RFL at Ns = N1/RFL) with the four-step
                // twiddle folded in.  Output m of butterfly jj is k1 = jj +
                // Ns m, and W_N^{n2 k1} = W_N^{n2 jj} W_N^{n2 Ns m}: the first
                // factor is common to the butterfly, so it joins the stage's
                // input twiddles W_N1^{jj q} (one phase per input,
                // W_N^{jj (n2 + N2 q)}), the second is wave-uniform (one
                // product per output).  Phases in exact 32-bit fixed point.
                FW::template run_head_tw<false, 1, F...>(v, wl, lane, tw16);
                constexpr int NsL = N1 / RFL;
                constexpr int LG1 = __builtin_ctz((unsigned)N1);
                const int LGN = __builtin_ctzll((unsigned long long)k.N);        // N = 2^LGN here
                const uint32_t A = (uint32_t)(n20 + wv) << (32 - LGN);           // n2 / N (2^-32 rev)
                cf U[RFL];
#pragma unroll
                for (int m = 1; m < RFL; ++m) U[m] = expi_rev(-fix32_to_rev(A * (uint32_t)(NsL * m)));
#pragma unroll
                for (int ib = 0; ib < E / RFL; ++ib) {
                    const uint32_t jj = (uint32_t)(lane + 64 * ib);              // < NsL
                    const uint32_t X0 = jj * A, S = jj << (32 - LG1);
                    cf *a = v + ib * RFL;
#pragma unroll
                    for (int q = 0; q < RFL; ++q) a[q] = cmul(a[q], expi_rev(-fix32_to_rev(X0 + (uint32_t)q * S)));
                    dft<RFL, false>(a);
#pragma unroll
                    for (int m = 1; m < RFL; ++m) a[m] = cmul(a[m], U[m]);
                }
            } else {
                FW::template run_tw<false, 1, F...>(v, wl, lane, tw16);
#pragma unroll
                for (int i = 0; i < E; ++i) {
                    int b0, k1;
                    FW::template where<RFL>(i, lane, b0, k1);
                    const uint32_t m = (uint32_t)(n20 + wv) * (uint32_t)k1;
                    float rev = (float)m * invN;
                    if (rev >= 0.5f) rev -= 1.0f;
                    v[i] = cmul(v[i], expi_rev(-rev));
                }
            }
            FW::template store<RFL>(v, wl, lane);
        } else {
            FF::template load<RF0>(v, lds, tid);
            __syncthreads();
            FF::template run_tw<false, 1, F...>(v, lds, tid, tw16);
#pragma unroll
            for (int i = 0; i < E; ++i) {
                int b, k1;
                FF::template where<RFL>(i, tid, b, k1);
                // (n20 + b) k1 < N1 N2 = N <= 2^24: exact in 32-bit and in float
                const uint32_t m = (uint32_t)(n20 + b) * (uint32_t)k1;
                float rev = (float)m * invN;
                if (rev >= 0.5f) rev -= 1.0f;
                v[i] = cmul(v[i], expi_rev(-rev));
            }
            FF::template store<RFL>(v, lds, tid);
        }
        __syncthreads();
        spill_block(k, lds, tid, pr, n20);
    }

    // The spill of a column block from LDS (natural k1 per column row):
    // 16-B stores of 4 columns per row k1, 32 consecutive rows per 32-lane group.
    __device__ static __forceinline__ void spill_block(const KP &k, const cf *lds, int tid, int pr, int64_t n20) {
        cf *Y = k.Yd + (int64_t)pr * pstride(k);
        const int64_t RP = rpitch(k);
        for (int it = tid; it < N1 * B / 4; it += T) {
            int k1, b4;
            if constexpr (B < 32 && N1 % 32 == 0) {
                // 32-lane groups: 32 consecutive rows of one 4-column group
                // (the lanes of a store instruction still cover whole row
                // segments, two lanes 32 apart per 64-B segment)
                const int g = it >> 5;
                b4 = (g % (B / 4)) * 4;
                k1 = (g / (B / 4)) * 32 + (it & 31);
            } else {
                k1 = it / (B / 4);
                b4 = (it - k1 * (B / 4)) * 4;
            }
            cf a0 = lds[LdsC::at(b4 + 0, k1)], a1 = lds[LdsC::at(b4 + 1, k1)];
            cf a2 = lds[LdsC::at(b4 + 2, k1)], a3 = lds[LdsC::at(b4 + 3, k1)];
            PSS_DASSERT((int64_t)k1 * RP + n20 + b4 + 4 <= pstride(k));
            float4 *dst = reinterpret_cast<float4 *>(Y + (int64_t)k1 * RP + n20 + b4);
            dst[0] = make_float4(a0.x, a0.y, a1.x, a1.y);
            dst[1] = make_float4(a2.x, a2.y, a3.x, a3.y);
        }
    }

    // Register columns (kRegCols): forward DFT of this thread's column n2
    // (x[n1] = z(n1 N2 + n2)), four-step twiddle W_N^{n2 k1}, spill row k1
    // at column n2.
    __device__ static __forceinline__ void reg_spill(const KP &k, cf (&x)[N1], int pr, int64_t n2) {
        static_assert(kRegCols, "register columns only");
        RegDft<N1, false>::run(x);
        const Buf Y(k.Yd + (int64_t)pr * pstride(k), (uint32_t)(pstride(k) * 8));
        const uint32_t RP = (uint32_t)rpitch(k);
        const float invN = k.invN;
#pragma unroll
        for (int k1 = 0; k1 < N1; ++k1) {
            // n2 k1 < N (exact in 32-bit and in float)
            float rev = (float)((uint32_t)n2 * (uint32_t)k1) * invN;
            if (rev >= 0.5f) rev -= 1.0f;
            const cf w = k1 ? cmul(x[k1], expi_rev(-rev)) : x[k1];
            Y.st2(w, ((uint32_t)k1 * RP + (uint32_t)n2) * 8u, 0u);
        }
    }
    // ... and back: spill column n2 times W_N^{-n2 k1}, inverse DFT
    // (unscaled), x[n1] = z(n1 N2 + n2) N.
    __device__ static __forceinline__ void reg_unspill(const KP &k, cf (&x)[N1], int pr, int64_t n2) {
        static_assert(kRegCols, "register columns only");
        const Buf Y(k.Yd + (int64_t)pr * pstride(k), (uint32_t)(pstride(k) * 8));
        const uint32_t RP = (uint32_t)rpitch(k);
        const float invN = k.invN;
#pragma unroll
        for (int k1 = 0; k1 < N1; ++k1) x[k1] = Y.ld2(((uint32_t)k1 * RP + (uint32_t)n2) * 8u, 0u);
#pragma unroll
        for (int k1 = 1; k1 < N1; ++k1) {
            float rev = (float)((uint32_t)n2 * (uint32_t)k1) * invN;
            if (rev >= 0.5f) rev -= 1.0f;
            x[k1] = cmul(x[k1], expi_rev(rev));
        }
        RegDft<N1, true>::run(x);
    }

    // Fold-mode fast passes (host-selected on the mixed-radix split: fold
    // source, chi2(df != 1) draws by the pair sampler, no injected draws, no
    // null in the epilogue).  Every lane owns one column n2 = n20 + lane and
    // keeps it in registers from the draws to the spill: no LDS at all.  The
    // pair sampler keys samples (2m, 2m + 1) -- columns (n2 & ~1, n2 | 1) of
    // one row -- so the lanes of a column pair split the draws by channel
    // (even lane: channel a, odd lane: channel b, both columns) and swap the
    // halves with one DPP move: every draw once, bitwise the values
    // source4 / epilogue4 produce (test_gpu_configs: fold fast == generic).
    __device__ static __forceinline__ void pair_draws(const Rng &g, uint32_t n, uint32_t cme, bool odd, float df,
                                                      float &va, float &vb) {
        float x0, x1;
        chi2_pair(g, n >> 1, cme, df, x0, x1);
        const float send = odd ? x0 : x1;          // even: a(n2 | 1); odd: b(n2 & ~1)
        const float recv = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0xB1, 0xF, 0xF, false));
        va = odd ? recv : x0;
        vb = odd ? x1 : recv;
    }
    __device__ static void passA_fold(const KP &k) {
        static_assert(kRegCols, "fold fast pass A: register columns");
        const int tid = threadIdx.x;
        int cbx, pr;
        xcd_block(cbx, pr);
        const int ra = 2 * pr - k.poff, rb = ra + 1;
        const bool hasa = ra >= 0, hasb = rb < k.p.nchan;
        const PssPipeline &p = k.p;
        const uint32_t n2 = (uint32_t)(cbx * B + tid), N2 = (uint32_t)k.N2;
        const uint32_t ca = (uint32_t)(p.chan0 + ra), cb = ca + 1u;
        const bool odd = (tid & 1) != 0;
        const Rng g(p.seed, p.call_gen, P_PULSE);
        const int last = p.prof_rows - 1;
        const int pra = (p.prof_rows == 1) ? 0 : min(max((int)ca - p.prof_row0, 0), last);
        const int prb = (p.prof_rows == 1) ? 0 : min(max((int)cb - p.prof_row0, 0), last);
        const float *pfa = p.prof + (int64_t)pra * p.nph, *pfb = p.prof + (int64_t)prb * p.nph;
        const uint32_t nph = (uint32_t)p.nph;
        const float dn = p.draw_norm, df = p.gen_df;
        cf x[N1];
        uint32_t b = n2 % nph;                       // profile bin of sample n1 N2 + n2
        const uint32_t db = N2 % nph;
        // (compile-time row index: a runtime-indexed x[] would live in scratch)
        static_for<0, N1>([&](auto IC) {
            constexpr int n1 = decltype(IC)::value;
            const uint32_t n = (uint32_t)n1 * N2 + n2;
            float va, vb;
            pair_draws(g, n, odd ? cb : ca, odd, df, va, vb);
            x[n1] = make_float2(hasa ? pfa[b] * va * dn : 0.f, hasb ? pfb[b] * vb * dn : 0.f);
            b += db;
            if (b >= nph) b -= nph;
        });
        reg_spill(k, x, pr, n2);
    }
    __device__ static void passC_fold(const KP &k) {
        static_assert(kRegCols, "fold fast pass C: register columns");
        const int tid = threadIdx.x;
        int cbx, pr;
        xcd_block(cbx, pr);
        const int ra = 2 * pr - k.poff, rb = ra + 1;
        const bool hasa = ra >= 0, hasb = rb < k.p.nchan;
        const PssPipeline &p = k.p;
        const uint32_t n2 = (uint32_t)(cbx * B + tid), N2 = (uint32_t)k.N2;
        const uint32_t ca = (uint32_t)(p.chan0 + ra), cb = ca + 1u;
        const bool odd = (tid & 1) != 0;
        const Rng g(p.seed, p.call_noise, P_NOISE);
        const float invN = k.invN, nn = p.noise_norm, df = p.noise_df;
        // The scaled column is staged in LDS, private to the lane (no
        // barrier): the noise loop may call the rare Marsaglia-Tsang retry,
        // and a whole column held in registers across those calls spills
        // (167 VGPRs of scratch at N1 = 30).
        __shared__ cf sg[N1 * B];                       // [n1][lane]
        {
            cf x[N1];
            reg_unspill(k, x, pr, n2);
#pragma unroll
            for (int n1 = 0; n1 < N1; ++n1) sg[n1 * B + tid] = make_float2(x[n1].x * invN, x[n1].y * invN);
        }
        float *oa = p.data + (int64_t)max(ra, 0) * p.ld, *ob = p.data + (int64_t)min(rb, p.nchan - 1) * p.ld;
#pragma unroll 2
        for (int n1 = 0; n1 < N1; ++n1) {
            const uint32_t n = (uint32_t)n1 * N2 + n2;
            float va, vb;
            pair_draws(g, n, odd ? cb : ca, odd, df, va, vb);
            const cf z = sg[n1 * B + tid];
            if (hasa) oa[n] = fmaf(nn, va, z.x);
            if (hasb) ob[n] = fmaf(nn, vb, z.y);
        }
    }

    // inverse column FFTs of one spilled pair block; result left in LDS in
    // natural order (LdsC::at(column, n1)), unscaled.  The load loop is
    // deliberately rolled: with every load of the block in flight at once
    // (64 KB per workgroup) the column passes overflow the XCD's L2 and the
    // half-line reads / 32-B output segments of neighbouring blocks stop
    // merging (PMC: +19% FETCH, +31% WRITE, pass C 17.6 -> 18.5 ms).
    __device__ static __forceinline__ void inv_block(const KP &k, const cf *Yp, int64_t n20, cf *lds, int tid) {
        __shared__ cf tw16[kTw16Size];
        tw16_fill(tw16, tid, T);     // read after the spill loads' barrier
        const int64_t N2 = k.N2;
        const float invN = k.invN;
        const Buf Y(Yp, (uint32_t)(pstride(k) * 8));   // one pair spill, < 2^28 bytes
        const uint32_t RP = (uint32_t)rpitch(k);
        const uint32_t s0 = (uint32_t)n20 * 8u;        // wave-uniform part of the offset
        {
#pragma unroll 1
        for (int it = tid; it < N1 * B / 4; it += T) {
            const int k1 = it / (B / 4);
            const int b4 = (it - k1 * (B / 4)) * 4;
            const uint32_t off = ((uint32_t)k1 * RP + (uint32_t)b4) * 8u;
            const float4 lo = Y.ld4(off, s0), hi = Y.ld4(off + 16u, s0);
            const cf a[4] = {make_float2(lo.x, lo.y), make_float2(lo.z, lo.w),
                             make_float2(hi.x, hi.y), make_float2(hi.z, hi.w)};
            // W^{m}, m = (n20 + b4 + i) k1 < N (exact in 32-bit and float):
            // W^{(n20 + b4) k1} (W^{k1})^i -- two native sincos per 4 points
            const uint32_t m0 = (uint32_t)(n20 + b4) * (uint32_t)k1;
            float r0 = (float)m0 * invN;
            if (r0 >= 0.5f) r0 -= 1.0f;
            float r1 = (float)k1 * invN;
            if (r1 >= 0.5f) r1 -= 1.0f;
            const cf w0 = expi_rev(r0), w1 = expi_rev(r1);
            const cf w2 = cmul(w1, w1);
            const cf tw[4] = {w0, cmul(w0, w1), cmul(w0, w2), cmul(w0, cmul(w2, w1))};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                lds[LdsC::at(b4 + i, k1)] = cmul(a[i], tw[i]);
            }
        }
        }
        __syncthreads();
        cf v[E];
        if constexpr (kWaveCols) {
            const int wv = tid >> 6, lane = tid & 63;
            cf *wl = lds + wv * LdsC::RS;
            FW::template load<RI0>(v, wl, lane);
            stage_sync<true>();
            FW::template run_tw<true, 1, I...>(v, wl, lane, tw16);
            FW::template store<RIL>(v, wl, lane);
        } else {
            FF::template load<RI0>(v, lds, tid);
            __syncthreads();
            FF::template run_tw<true, 1, I...>(v, lds, tid, tw16);
            FF::template store<RIL>(v, lds, tid);
        }
        __syncthreads();
    }

    // C: inverse column FFTs of the data pair, then the epilogues of channels
    // a, b straight from LDS (delayed-null decisions from the mask table).
    __device__ static void passC(const KP &k) {
        __shared__ __align__(128) cf lds[B * LdsC::RS];   // (128-B aligned: the FFT's byte-address exchanges)
        const int tid = threadIdx.x;
        int cbx, pr;
        xcd_block(cbx, pr);
        const int ra = 2 * pr - k.poff, rb = ra + 1;
        const bool hasa = ra >= 0, hasb = rb < k.p.nchan;
        const int64_t n20 = (int64_t)cbx * B;
        const bool mask = k.mtab != 0;
        const float invN = k.invN;
        if constexpr (kRegCols) {
            cf x[N1];
            reg_unspill(k, x, pr, n20 + tid);
#pragma unroll
            for (int n1 = 0; n1 < N1; ++n1) lds[LdsC::at(tid, n1)] = x[n1];
            __syncthreads();
        } else {
            inv_block(k, k.Yd + (int64_t)pr * pstride(k), n20, lds, tid);
        }
#pragma unroll 1
        for (int it = tid; it < N1 * B / 4; it += T) {
            const int n1 = it / (B / 4);
            const int b4 = (it - n1 * (B / 4)) * 4;
            const int64_t n = n1 * k.N2 + n20 + b4;
            float da[4], db[4], ma[4], mb[4];
            const uint32_t ha = (mask && hasa) ? mask_bits4<B, N1>(k, ra, cbx, n1, b4) : 0u;
            const uint32_t hb = (mask && hasb) ? mask_bits4<B, N1>(k, rb, cbx, n1, b4) : 0u;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const cf z = lds[LdsC::at(b4 + i, n1)];
                da[i] = z.x * invN;
                db[i] = z.y * invN;
                ma[i] = ((ha >> i) & 1u) ? 2.0f : 0.0f;
                mb[i] = ((hb >> i) & 1u) ? 2.0f : 0.0f;
            }
            if (hasa) epilogue4(k, ra, n, 4, da, ma, false);
            if (hasb) epilogue4(k, rb, n, 4, db, mb, false);
        }
    }

    // C, fast path (host-selected: Philox draws with df = 1 for the noise, no
    // injected draws, no observe() copy).  Bitwise equal to passC: every
    // sample is stored as signal + noise; a delayed null's samples are
    // rewritten afterwards by k_null_fix_list (fusing the table lookups here
    // measured 27.0 ms against 16.6 + 2.5 for pass C + fix-up, round 2).
    // C, fast path with register-resident columns (C5's 2048-point columns,
    // 16 columns per 512-thread workgroup: 64-B output segments per channel
    // row instead of 32; tools/seg_bw.hip: 64-B write segments run at 5.2
    // TB/s against 3.1 for 32 B).  16 columns of 2048 rows are 256 KB, so
    // they cannot all sit in LDS: each wave keeps its columns in registers
    // between three LDS phases --
    // (1) the spill rows in two halves of 512 (256-B row segments, twiddled as
    // in inv_block) staged in LDS and picked up into the FFT input mapping,
    // (2) the two wave-local inverse FFTs one after the other through the
    // wave's own LDS row, (3) each channel's scaled outputs staged as
    // [n1][33] floats and stored as whole 128-B row segments with the noise.
    // Bitwise the values of passC_fast (same twiddles, FFT and epilogue).
    __device__ static void passC_fast32(const KP &k) {
        static_assert((N1 == 1024 || N1 == 2048) && (T == 1024 || T == 512) && B % (T / 64) == 0 &&
                      kWaveCols == false, "register-resident wide pass C: 2^m columns of 1024 / 2048");
        constexpr int NW = T / 64, CPW = B / NW;        // waves, columns per wave
        constexpr int E1 = N1 / 64;                     // values per lane of one column
        constexpr int H = N1 / 2;                       // rows per load half
        constexpr int RSH = H + H / 16 + 1;             // padded pitch of a half column (odd)
        constexpr int OSP = B + 1;                      // staging pitch (floats)
        using LW = Lds<N1, -1>;                         // FFT rows: padded, as passC_fast's
        using FWC = Fft<N1, 1, 64, true, -1>;
        constexpr int RI0 = FWC::template first<I...>();
        constexpr int LRI = N1 / RI0;                   // input mapping: v[ib RI0 + q] = lane + 64 ib + LRI q
        constexpr int B1 = B * RSH * 8, B2 = NW * LW::RS * 8, B3 = N1 * OSP * 4;
        constexpr int BUF = (B1 > B2 ? B1 : B2) > B3 ? (B1 > B2 ? B1 : B2) : B3;
        __shared__ __align__(16) char smem[BUF];
        __shared__ cf tw16[kTw16Size];
        const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
        tw16_fill(tw16, tid, T);
        int cbx, pr;
        xcd_block(cbx, pr);
        const int ra = 2 * pr - k.poff, rb = ra + 1;
        const bool hasa = ra >= 0, hasb = rb < k.p.nchan;
        const int64_t N2 = k.N2;
        const PssPipeline &p = k.p;
        const float invN = k.invN, nn = p.noise_norm;
        const int64_t n20 = (int64_t)cbx * B;
        const Buf Y(k.Yd + (int64_t)pr * pstride(k), (uint32_t)(pstride(k) * 8));
        const uint32_t RP = (uint32_t)rpitch(k);
        cf *hb = reinterpret_cast<cf *>(smem);
        cf v[CPW][E1];
        // (1) spill rows, two halves
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (h) __syncthreads();                     // the first half has been picked up
#pragma unroll 1
            for (int it = tid; it < H * B / 4; it += T) {
                const int k1l = it / (B / 4), b4 = (it - k1l * (B / 4)) * 4;
                const int k1 = h * H + k1l;
                const uint32_t off = ((uint32_t)k1 * RP + (uint32_t)b4) * 8u, so = (uint32_t)n20 * 8u;
                const float4 lo = Y.ld4(off, so), hi = Y.ld4(off + 16u, so);
                const cf a[4] = {make_float2(lo.x, lo.y), make_float2(lo.z, lo.w),
                                 make_float2(hi.x, hi.y), make_float2(hi.z, hi.w)};
                // the twiddles of inv_block, bit for bit
                const uint32_t m0 = (uint32_t)(n20 + b4) * (uint32_t)k1;
                float r0 = (float)m0 * invN;
                if (r0 >= 0.5f) r0 -= 1.0f;
                float r1 = (float)k1 * invN;
                if (r1 >= 0.5f) r1 -= 1.0f;
                const cf w0 = expi_rev(r0), w1 = expi_rev(r1);
                const cf w2 = cmul(w1, w1);
                const cf tw[4] = {w0, cmul(w0, w1), cmul(w0, w2), cmul(w0, cmul(w2, w1))};
#pragma unroll
                for (int i = 0; i < 4; ++i) hb[(b4 + i) * RSH + k1l + (k1l >> 4)] = cmul(a[i], tw[i]);
            }
            __syncthreads();
            // the FFT input mapping: register i = ib RI0 + q holds position
            // lane + 64 ib + LRI q (the half it lies in is compile-time)
#pragma unroll
            for (int i = 0; i < E1; ++i) {
                const int pc = 64 * (i / RI0) + LRI * (i % RI0);      // position minus lane
                if (pc / H != h) continue;
                const int pl = lane + pc - h * H;
#pragma unroll
                for (int c = 0; c < CPW; ++c) v[c][i] = hb[(wv + NW * c) * RSH + pl + (pl >> 4)];
            }
        }
        __syncthreads();
        // (2) the inverse column FFTs through the wave's own LDS row
        {
            cf *wl = reinterpret_cast<cf *>(smem) + wv * LW::RS;
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                if (c) stage_sync<true>();
                FWC::template run_tw<true, 1, I...>(v[c], wl, lane, tw16);
            }
        }
        // (3) per channel: stage the scaled outputs, store rows with the noise
        constexpr int RIL = FWC::template last_of<I...>();
        float *stg = reinterpret_cast<float *>(smem);
        const uint32_t ca = (uint32_t)(p.chan0 + ra), cb = ca + 1u;
        const Rng gn(p.seed, p.call_noise, P_NOISE);
        const uint32_t rbytes = (uint32_t)(k.N * 4);
#pragma unroll
        for (int ch = 0; ch < 2; ++ch) {
            __syncthreads();                            // FFT rows / previous channel's staging free
#pragma unroll
            for (int i = 0; i < E1; ++i) {
                int bb, pos;
                FWC::template where<RIL>(i, lane, bb, pos);
#pragma unroll
                for (int c = 0; c < CPW; ++c) stg[pos * OSP + wv + NW * c] = (ch ? v[c][i].y : v[c][i].x) * invN;
            }
            __syncthreads();
            const bool has = ch ? hasb : hasa;
            if (!has) continue;                         // (uniform)
            const uint32_t c = ch ? cb : ca;
            const Buf o(p.data + (int64_t)(ch ? rb : ra) * p.ld, rbytes);
#pragma unroll
            for (int t = 0; t < N1 * B / 4 / T; ++t) {
                const int it = tid + t * T;
                const int n1 = it / (B / 4), c4 = (it - n1 * (B / 4)) * 4;
                const uint32_t n = (uint32_t)(n1 * (int)N2) + (uint32_t)n20 + (uint32_t)c4;
                const float4 x = chi2_1x4(gn.bits(n >> 2, c, 0u));
                const float *sr = stg + n1 * OSP + c4;
                o.st4(fmaf(nn, x.x, sr[0]), fmaf(nn, x.y, sr[1]), fmaf(nn, x.z, sr[2]), fmaf(nn, x.w, sr[3]),
                      n * 4u, 0);
            }
        }
    }

    __device__ static void passC_fast(const KP &k) {
        static_assert(kItemsExact, "fast pass C: whole items per thread");
        __shared__ __align__(128) cf lds[B * LdsC::RS];
        const int tid = threadIdx.x;
        int cbx, pr;
        xcd_block(cbx, pr);
        const int ra = 2 * pr - k.poff, rb = ra + 1;
        const bool hasa = ra >= 0, hasb = rb < k.p.nchan;
        const int64_t N2 = k.N2;
        const PssPipeline &p = k.p;
        const float invN = k.invN, nn = p.noise_norm;
        const uint32_t ca = (uint32_t)(p.chan0 + ra), cb = ca + 1u;
        const Rng gn(p.seed, p.call_noise, P_NOISE);
        const uint32_t rbytes = (uint32_t)(k.N * 4);
        const Buf oa(p.data + (int64_t)max(ra, 0) * p.ld, rbytes), ob(p.data + (int64_t)min(rb, p.nchan - 1) * p.ld, rbytes);
        const int64_t n20 = (int64_t)cbx * B;
        inv_block(k, k.Yd + (int64_t)pr * pstride(k), n20, lds, tid);
        float acc[ITEMS][2][4];
#pragma unroll
        for (int t = 0; t < ITEMS; ++t) {
            const int it = tid + t * T;
            const int n1 = it / (B / 4);
            const int b4 = (it - n1 * (B / 4)) * 4;
            const uint32_t n = (uint32_t)(n1 * (int)N2) + (uint32_t)n20 + (uint32_t)b4;   // N <= 2^24
            const float4 xa = chi2_1x4(gn.bits(n >> 2, ca, 0u));
            const float4 xb = chi2_1x4(gn.bits(n >> 2, cb, 0u));
            const float na[4] = {xa.x, xa.y, xa.z, xa.w}, nb[4] = {xb.x, xb.y, xb.z, xb.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const cf z = lds[LdsC::at(b4 + i, n1)];
                acc[t][0][i] = fmaf(nn, na[i], z.x * invN);
                acc[t][1][i] = fmaf(nn, nb[i], z.y * invN);
            }
        }
        // (a delayed null's samples are rewritten afterwards: k_null_fix_list)
#pragma unroll
        for (int t = 0; t < ITEMS; ++t) {
            const int it = tid + t * T;
            const int n1 = it / (B / 4);
            const int b4 = (it - n1 * (B / 4)) * 4;
            const uint32_t off = ((uint32_t)(n1 * (int)N2) + (uint32_t)n20 + (uint32_t)b4) * 4u;
            if (hasa) oa.st4(acc[t][0][0], acc[t][0][1], acc[t][0][2], acc[t][0][3], off, 0);
            if (hasb) ob.st4(acc[t][1][0], acc[t][1][1], acc[t][1][2], acc[t][1][3], off, 0);
        }
    }

    // Mask table build: inverse column FFTs of node pair `blockIdx.y`, stored
    // (scaled) as node rows nodes[2 pr], nodes[2 pr + 1].
    __device__ static void node_col(const KP &k, float *nodes) {
        __shared__ __align__(128) cf lds[B * LdsC::RS];   // (128-B aligned: the FFT's byte-address exchanges)
        const int tid = threadIdx.x;
        int cbx, pr;
        xcd_block(cbx, pr);
        const int64_t n20 = (int64_t)cbx * B;
        const float invN = k.invN;
        inv_block(k, k.Ym + (int64_t)pr * pstride(k), n20, lds, tid);
        float *ra = nodes + (int64_t)(2 * pr) * k.N, *rb = ra + k.N;
        for (int it = tid; it < N1 * B / 4; it += T) {
            const int n1 = it / (B / 4);
            const int b4 = (it - n1 * (B / 4)) * 4;
            const int64_t n = n1 * k.N2 + n20 + b4;
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const cf z = lds[LdsC::at(b4 + i, n1)];
                a[i] = z.x * invN;
                b[i] = z.y * invN;
            }
            *reinterpret_cast<float4 *>(ra + n) = make_float4(a[0], a[1], a[2], a[3]);
            *reinterpret_cast<float4 *>(rb + n) = make_float4(b[0], b[1], b[2], b[3]);
        }
    }
};

template <typename C, int T>
__global__ __launch_bounds__(T) void k_pairA(KP k) { C::template passA<false>(k); }
template <typename C, int T, bool SHARED>
__global__ __launch_bounds__(T) void k_pairA_fast(KP k) { C::template passA<true, SHARED>(k); }
template <typename C, int T>
__global__ __launch_bounds__(T) void k_pairC(KP k) { C::passC(k); }
template <typename C, int T>
__global__ __launch_bounds__(T) void k_pairC_fast(KP k) { C::passC_fast(k); }
template <typename C, int T>
__global__ __launch_bounds__(T, T == 512 ? 2 : 4) void k_pairC_fast32(KP k) { C::passC_fast32(k); }
template <typename C, int T>
__global__ __launch_bounds__(T) void k_node_col(KP k, float *nodes) { C::node_col(k, nodes); }
// (4 waves per SIMD for columns up to 30: the compiler would otherwise keep
// every row's draws in flight at once, 210 VGPRs for N1 = 30)
template <typename C, int T>
__global__ __launch_bounds__(T, C::kFoldWaves) void k_pairA_fold(KP k) { C::passA_fold(k); }
template <typename C, int T>
__global__ __launch_bounds__(T, C::kFoldWavesC) void k_pairC_fold(KP k) { C::passC_fold(k); }


// Node ramps of the mask table: f_j = (t_j + 1)/2 at the Chebyshev points
// t_j = cos(pi (j + 1/2) / KCH); ramp word f_j / N * 2^64, Nyquist cos(pi f_j).
__global__ void k_node_params(uint64_t *ramp, float *nyq, int L) {
    const int j = threadIdx.x;
    if (j < KCH) {
        const double t = cospi((j + 0.5) / KCH);
        const double f = 0.5 * (t + 1.0);
        ramp[j] = (uint64_t)ldexp(f, 64 - L);
        nyq[j] = (float)cospi(f);
    }
}

// Per position p: Chebyshev coefficients of M(p, t) from the KCH node values,
// classification (never / always / depends-on-f nulled) with the bound
// |M - c0| <= sum_{n>=1} |c_n| on t in [-1, 1], and compaction of the
// coefficients of the f-dependent positions (wave ballot + one atomic per
// wave; positions are self-describing, so the atomic order does not matter).
__global__ __launch_bounds__(256) void k_mask_table(const float *nodes, int64_t N, uint2 *bits,
                                                    uint32_t *base, float *coef, uint32_t *counter) {
    __shared__ float T[KCH * KCH];
    if (threadIdx.x < KCH * KCH) {
        const int n = threadIdx.x / KCH, j = threadIdx.x - n * KCH;
        T[threadIdx.x] = (float)(cospi((double)n * (j + 0.5) / KCH) * (n ? 2.0 : 1.0) / KCH);
    }
    __syncthreads();
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // N % 256 == 0
    float v[KCH], c[KCH];
#pragma unroll
    for (int j = 0; j < KCH; ++j) v[j] = nodes[(int64_t)j * N + p];
    float S = 0.f;
#pragma unroll
    for (int n = 0; n < KCH; ++n) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < KCH; ++j) s = fmaf(T[n * KCH + j], v[j], s);
        c[n] = s;
        if (n) S += fabsf(s);
    }
    // margin covers the fp32 evaluation error of cheb_eval (~1e-6 sum|c|)
    const float eps = 1e-3f + 4e-6f * (fabsf(c[0]) + S);
    const bool hi = c[0] - S > 1.0f + eps;
    const bool amb = !hi && !(c[0] + S < 1.0f - eps);
    const uint64_t ab = __ballot(amb), hb = __ballot(hi);
    const int lane = threadIdx.x & 63;
    uint32_t b0 = 0;
    if (lane == 0 && ab) b0 = atomicAdd(counter, (uint32_t)__popcll(ab));
    b0 = __shfl(b0, 0);
    if (lane == 0) {   // this wave's 64 positions = table words p/32, p/32 + 1
        bits[p >> 5] = make_uint2((uint32_t)hb, (uint32_t)ab);
        bits[(p >> 5) + 1] = make_uint2((uint32_t)(hb >> 32), (uint32_t)(ab >> 32));
        base[p >> 5] = b0;
        base[(p >> 5) + 1] = b0 + (uint32_t)__popc((uint32_t)ab);
    }
    if (amb) {
        // root record (root_hit): where the fp32 Clenshaw value crosses 1,
        // on a certified scan grid (see root_hit)
        const float4 q[3] = {make_float4(c[0], c[1], c[2], c[3]), make_float4(c[4], c[5], c[6], c[7]),
                             make_float4(c[8], c[9], c[10], c[11])};
        float D2 = 0.f;                              // max |g''| on [-1, 1] (Markov)
#pragma unroll
        for (int n = 2; n < KCH; ++n) {
            const float n2 = (float)(n * n);
            D2 = fmaf(n2 * (n2 - 1.0f) * (1.0f / 3.0f), fabsf(c[n]), D2);
        }
        const float err = 4e-6f * (fabsf(c[0]) + S);  // fp32 Clenshaw error bound (as eps)
        constexpr int NG = 256;
        constexpr float H = 2.0f / NG;
        float rt[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) rt[i] = INFINITY;
        float gprev = cheb_eval_r(q, -1.0f) - 1.0f;
        bool prev = gprev > 0.0f;
        const bool s0 = prev;
        bool cert = true;
        int cnt = 0;
        float tprev = -1.0f;
        for (int jg = 1; jg <= NG; ++jg) {
            const float tg = -1.0f + (float)jg * H;
            const float g = cheb_eval_r(q, tg) - 1.0f;
            const bool cur = g > 0.0f;
            if (cur != prev) {
                cert = cert && (fabsf(g - gprev) - 2.0f * err > D2 * H * H);   // one flip only
                float lo = tprev, hi = tg;            // decision prev at lo, cur at hi
                for (int it = 0; it < 24; ++it) {
                    const float mid = 0.5f * (lo + hi);
                    if ((cheb_eval_r(q, mid) > 1.0f) == prev) lo = mid; else hi = mid;
                }
#pragma unroll
                for (int i = 0; i < 10; ++i) if (i == cnt) rt[i] = lo;
                ++cnt;
            } else {
                // no flip: g stays within D2 H^2 / 8 of the chord between the
                // cell's ends, whose values share a sign
                cert = cert && (fminf(fabsf(g), fabsf(gprev)) - err > D2 * H * H * 0.125f);
            }
            prev = cur;
            gprev = g;
            tprev = tg;
        }
        const uint32_t idx = b0 + (uint32_t)__popcll(ab & ((1ull << lane) - 1ull));
        float4 *dst = reinterpret_cast<float4 *>(coef + (int64_t)idx * KREC);
        if (cert && cnt <= 10) {
            dst[0] = make_float4((float)cnt, s0 ? 1.0f : 0.0f, rt[0], rt[1]);
            dst[1] = make_float4(rt[2], rt[3], rt[4], rt[5]);
            dst[2] = make_float4(rt[6], rt[7], rt[8], rt[9]);
        } else {
            dst[0] = make_float4(-1.0f, 0.0f, 0.0f, 0.0f);
            dst[1] = q[0];
            dst[2] = q[1];
            dst[3] = q[2];
        }
    }
}

// ---------------------------------------------------------------------------
// path 3: direct DFT fallback for even N that are not handled above.
//   W1[row][n] = source (complex), W2[row][k] = DFT(W1) * ramp, then inverse
//   DFT + epilogue.  O(N^2); LDS-tiled over the summation index.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fb_source(KP k) {
    const int r = blockIdx.y;
    cf *W1 = reinterpret_cast<cf *>(k.p.work) + (int64_t)r * k.N;
    const int64_t items = (k.N + 3) >> 2;
    const bool re_in = k.p.data_in_fft != 0;
    for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < items;
         it += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n0 = it << 2;
        const int cnt = (int)min((int64_t)4, k.N - n0);
        float re[4], im[4];
        source4(k, r, n0, cnt, re, im, re_in);
        for (int i = 0; i < cnt; ++i) W1[n0 + i] = make_float2(re[i], im[i]);
    }
}

// exp(-2 pi i m / N) for m in [0, N), double-precision angles (fallback path)
__global__ void k_fb_twiddles(KP k) {
    cf *tw = reinterpret_cast<cf *>(k.p.work) + (int64_t)2 * k.p.nchan * k.N;
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < k.N;
         m += (int64_t)gridDim.x * blockDim.x) {
        double s, c;
        sincospi(-2.0 * (double)m / (double)k.N, &s, &c);
        tw[m] = make_float2((float)c, (float)s);
    }
}

template <bool INV>
__global__ __launch_bounds__(256) void k_fb_dft(KP k) {
    __shared__ cf tile[1024];
    const int r = blockIdx.y;
    const int64_t N = k.N;
    const cf *in = reinterpret_cast<const cf *>(k.p.work) + (int64_t)(INV ? k.p.nchan + r : r) * N;
    const cf *tw = reinterpret_cast<const cf *>(k.p.work) + (int64_t)2 * k.p.nchan * N;
    const int64_t kout = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double accr = 0.0, acci = 0.0;
    // twiddle index m = (kout * n) mod N, advanced incrementally (exact)
    const int64_t kk = kout < N ? kout : 0;
    for (int64_t base = 0; base < N; base += 1024) {
        const int cnt = (int)min((int64_t)1024, N - base);
        __syncthreads();
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) tile[i] = in[base + i];
        __syncthreads();
        int64_t m = (kk * base) % N;
        for (int i = 0; i < cnt; ++i) {
            cf w = tw[m];
            if (INV) w.y = -w.y;
            const cf x = tile[i];
            accr += (double)x.x * w.x - (double)x.y * w.y;
            acci += (double)x.x * w.y + (double)x.y * w.x;
            m += kk;
            if (m >= N) m -= N;
        }
    }
    if (kout >= N) return;
    if (!INV) {
        cf z = apply_ramp(k, r, kout, make_float2((float)accr, (float)acci));
        reinterpret_cast<cf *>(k.p.work)[(int64_t)(k.p.nchan + r) * N + kout] = z;
    } else {
        // stash the inverse result in W1 (no longer needed) for the epilogue
        reinterpret_cast<cf *>(k.p.work)[(int64_t)r * N + kout] =
            make_float2((float)(accr / (double)N), (float)(acci / (double)N));
    }
}

__global__ __launch_bounds__(256) void k_fb_epilogue(KP k) {
    const int r = blockIdx.y;
    const cf *W1 = reinterpret_cast<const cf *>(k.p.work) + (int64_t)r * k.N;
    const int64_t items = (k.N + 3) >> 2;
    const bool re_in = k.p.data_in_fft != 0;
    for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < items;
         it += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n0 = it << 2;
        const int cnt = (int)min((int64_t)4, k.N - n0);
        float pre[4] = {0, 0, 0, 0}, msk[4] = {0, 0, 0, 0};
        for (int i = 0; i < cnt; ++i) { pre[i] = W1[n0 + i].x; msk[i] = W1[n0 + i].y; }
        epilogue4(k, r, n0, cnt, pre, msk, !re_in);
    }
}

// ---------------------------------------------------------------------------
// Delayed null on the packed (direct / Bluestein) paths, decided in float64.
// These paths carry the box row through the channel's complex transform as
// its imaginary part, so the fp32 mask shares the error of the data (fold-mode
// rows peak at ~1e4; the boxes are chi2(Nfold) values of that size themselves)
// and a few percent of the samples sit within that error of the threshold 1.
// For those samples (|mask - 1| < max(1e-3, 3e-5 x the row's largest |value|),
// a generous multiple of the transform's measured ~2e-6 relative error) the
// mask is re-evaluated in float64 from the box row's spectrum B(k) (once per
// run, channel independent):
//   m(n) = ( B_0 + 2 sum_{0<k<N/2} Re(B_k e^{2 pi i k (n/N - s)}) + B_{N/2} nyq (-1)^n ) / N,
// s = the channel's ramp (frac(delay/N)), nyq its mask Nyquist factor -- the
// reference's shift_t of the box row by the total delay (pulsar.py:306-330,
// utils.py:17-59) -- and its decision m > 1 replaces the fp32 one (encoded as
// mask 2 / 0 for the epilogue).  The candidates are first compacted into a
// list (k_null_cands), then one wave per candidate (k_null_refine_list, the
// waves striding over the list: candidates cluster at the box edges, so a
// wave per 64 samples left a few waves with most of the work -- C4's
// geometry with a null: 26.7 ms of refine), the bins split over the lanes in
// four interleaved phasor recurrences (independent chains: the recurrence's
// float64 latency no longer serialises the loop), a wave sum.  A list that
// would overflow its capacity falls back to the per-sample kernel
// (k_null_refine) for the whole run.  The box spectrum is summed in kBsParts
// sample ranges (all CUs busy; all-zero 1024-sample tiles skipped), then
// reduced in a fixed order (run to run the same bits).
// Even N <= kRefineMaxN (the O(N x nnz) box spectrum), no scattering tail
// (an extension whose packed path also filters the mask).
// ---------------------------------------------------------------------------
static constexpr int64_t kRefineMaxN = 1 << 17;
static constexpr int kBsParts = 16;
// refine candidate list capacity (entries of 8 B): 1/8 of the samples + 64 Ki
// (C4's fold-mode geometry with a null has ~7 % candidates: its boxes are
// chi2(Nfold ~ 1e4) values, so the band is ~0.3 wide and the boxes' Gibbs
// ringing crosses it often)
static inline int64_t refine_cap(int32_t nchan, int64_t N) {
    const int64_t all = (int64_t)nchan * N;
    return std::min<int64_t>(all, all / 8 + 65536);
}

__global__ __launch_bounds__(256) void k_tw64(int64_t N, double2 *tw) {
    for (int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x; n < N; n += (int64_t)gridDim.x * 256) {
        double sn, cs;
        sincospi(2.0 * (double)n / (double)N, &sn, &cs);
        tw[n] = make_double2(cs, sn);                    // e^{+2 pi i n / N}
    }
}

// partial box spectra: part[p][k] = sum_{n in range p} box[n] e^{-2 pi i k n / N},
// k <= N/2, float64 (grid: bins / 256 x kBsParts sample ranges; the tile
// loop is uniform over the workgroup, so skipping zero tiles / samples does
// not diverge)
__global__ __launch_bounds__(256) void k_null_bspec(const float *box, int64_t N, const double2 *tw, double2 *part) {
    __shared__ float tile[1024];
    const int64_t K = N / 2 + 1;
    const int64_t kb = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t kk = kb < K ? kb : 0;
    const int64_t n0 = N * (int64_t)blockIdx.y / kBsParts, n1 = N * ((int64_t)blockIdx.y + 1) / kBsParts;
    double re = 0.0, im = 0.0;
    for (int64_t base = n0; base < n1; base += 1024) {
        const int cnt = (int)min((int64_t)1024, n1 - base);
        __syncthreads();
        int nz = 0;
        for (int i = threadIdx.x; i < cnt; i += 256) {
            const float b = box[base + i];
            tile[i] = b;
            nz |= b != 0.0f;
        }
        if (!__syncthreads_or(nz)) continue;          // (the barrier also orders the tile)
        int64_t m = (kk * base) % N;
        for (int i = 0; i < cnt; ++i) {
            const float b = tile[i];
            if (b != 0.0f) {
                const double2 w = tw[m];
                re += (double)b * w.x;
                im -= (double)b * w.y;
            }
            m += kk;
            if (m >= N) m -= N;
        }
    }
    if (kb < K) part[(int64_t)blockIdx.y * K + kb] = make_double2(re, im);
}

// B_k = the parts summed in a fixed order
__global__ __launch_bounds__(256) void k_null_bsum(const double2 *part, int64_t K, double2 *B) {
    const int64_t kb = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (kb >= K) return;
    double re = 0.0, im = 0.0;
#pragma unroll
    for (int p = 0; p < kBsParts; ++p) {
        const double2 v = part[(int64_t)p * K + kb];
        re += v.x;
        im += v.y;
    }
    B[kb] = make_double2(re, im);
}

// per row: the largest |value| of the packed inverse (data and mask parts),
// the scale of its fp32 error (mx zeroed by the host; positive floats order
// as their bit patterns)
__global__ __launch_bounds__(256) void k_row_absmax(const cf *W1, int64_t N, unsigned int *mx) {
    const int r = blockIdx.y;
    float v = 0.0f;
    for (int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x; n < N; n += (int64_t)gridDim.x * 256) {
        const cf z = W1[(int64_t)r * N + n];
        v = fmaxf(v, fmaxf(fabsf(z.x), fabsf(z.y)));
    }
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    if ((threadIdx.x & 63) == 0) atomicMax(mx + r, __float_as_uint(v));
}

// the float64 mask value m(n) at sample ns of channel r; wave-wide (every lane
// of the wave calls it for the same (r, ns)), the result valid in every lane
__device__ __forceinline__ double refine_mask(const KP &k, const double2 *B, int r, int64_t ns, int lane) {
    const int64_t N = k.N, H = N / 2;
    const double ramp = (double)k.p.ramp[r] * 5.421010862427522e-20;     // 2^-64
    // per-bin phase step (revolutions): n/N - s
    double phi = (double)ns / (double)N - ramp;
    phi -= floor(phi);
    // lane's bins k = 1 + lane + 64 j in four chains (j mod 4), each a
    // phasor recurrence of step e^{2 pi i 256 phi}
    double sn[4], cs[4], acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        sincospi(2.0 * phi * (double)(1 + lane + 64 * c), &sn[c], &cs[c]);
        acc[c] = 0.0;
    }
    double s256, c256;
    sincospi(2.0 * phi * 256.0, &s256, &c256);
    for (int64_t kb = 1 + lane; kb < H; kb += 256) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int64_t kc = kb + 64 * c;
            const double2 b = B[kc < H ? kc : 0];
            const double f = kc < H ? 1.0 : 0.0;
            acc[c] = fma(f * b.x, cs[c], fma(-f * b.y, sn[c], acc[c]));
            const double t = cs[c] * c256 - sn[c] * s256;
            sn[c] = cs[c] * s256 + sn[c] * c256;
            cs[c] = t;
        }
    }
    double a = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    double m = B[0].x + 2.0 * a;
    if (2 * H == N) m += B[H].x * (double)k.p.nyq_im[r] * ((ns & 1) ? -1.0 : 1.0);
    return m / (double)N;
}

static __device__ __forceinline__ bool refine_cand(const cf *z, int64_t n, int64_t N, float band) {
    return n < N && fabsf(z[n < N ? n : 0].y - 1.0f) < band;
}

// candidates of every row into the list (entry = r << 32 | n; order free:
// each entry's decision is computed on its own)
__global__ __launch_bounds__(256) void k_null_cands(KP k, const cf *W1, const unsigned int *mx,
                                                   unsigned long long *list, unsigned int *cnt, int64_t cap) {
    const int r = blockIdx.y, lane = threadIdx.x & 63;
    const int64_t N = k.N;
    const float band = fmaxf(1e-3f, 3e-5f * __uint_as_float(mx[r]));
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool cand = refine_cand(W1 + (int64_t)r * N, n, N, band);
    const uint64_t m = __ballot(cand);
    if (!m) return;
    unsigned int b0 = 0;
    if (lane == 0) b0 = atomicAdd(cnt, (unsigned int)__popcll(m));
    b0 = __shfl(b0, 0);
    if (cand) {
        const int64_t idx = (int64_t)b0 + __popcll(m & ((1ull << lane) - 1ull));
        if (idx < cap) list[idx] = ((unsigned long long)r << 32) | (unsigned long long)n;
    }
}

// four candidates per wave, sixteen per workgroup: the box spectrum goes
// through LDS in 1024-bin tiles that the workgroup's 16 candidates share,
// and every bin serves four phasor recurrences per wave (the candidates'
// independent chains).  A lane's bins k = 1 + lane + 64 j in order, as the
// per-sample kernel walks them.
__global__ __launch_bounds__(256) void k_null_refine_list(KP k, cf *W1, const double2 *B,
                                                         const unsigned long long *list, const unsigned int *cnt,
                                                         int64_t cap) {
    constexpr int C = 4, TB = 1024;
    __shared__ double2 tile[TB];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t total = min((int64_t)*cnt, cap);
    const int64_t N = k.N, H = N / 2;
    for (int64_t g0 = (int64_t)blockIdx.x * 16; g0 < total; g0 += (int64_t)gridDim.x * 16) {
        const int64_t e0 = g0 + wv * C;
        int r[C];
        int64_t ns[C];
        double sn[C], cs[C], s64[C], c64[C], acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int64_t e = e0 + c < total ? e0 + c : g0;           // (a repeat of g0: not written)
            const unsigned long long v = list[e];
            r[c] = (int)(v >> 32);
            ns[c] = (int64_t)(v & 0xffffffffull);
            double phi = (double)ns[c] / (double)N - (double)k.p.ramp[r[c]] * 5.421010862427522e-20;
            phi -= floor(phi);
            sincospi(2.0 * phi * (double)(1 + lane), &sn[c], &cs[c]);
            sincospi(2.0 * phi * 64.0, &s64[c], &c64[c]);
            acc[c] = 0.0;
        }
        for (int64_t base = 1; base < H; base += TB) {
            __syncthreads();                                  // the previous tile is consumed
            for (int i = threadIdx.x; i < TB; i += 256)
                tile[i] = base + i < H ? B[base + i] : make_double2(0.0, 0.0);
            __syncthreads();
            const int cntb = (int)min((int64_t)TB, H - base);
            for (int i = lane; i < cntb; i += 64) {
                const double2 b = tile[i];
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    acc[c] = fma(b.x, cs[c], fma(-b.y, sn[c], acc[c]));
                    const double t = cs[c] * c64[c] - sn[c] * s64[c];
                    sn[c] = cs[c] * s64[c] + sn[c] * c64[c];
                    cs[c] = t;
                }
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            double a = acc[c];
            for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
            double m = B[0].x + 2.0 * a;
            if (2 * H == N) m += B[H].x * (double)k.p.nyq_im[r[c]] * ((ns[c] & 1) ? -1.0 : 1.0);
            m /= (double)N;
            if (lane == 0 && e0 + c < total) W1[(int64_t)r[c] * N + ns[c]].y = m > 1.0 ? 2.0f : 0.0f;
        }
    }
}

// the per-sample form: only when the candidate list overflowed its capacity
__global__ __launch_bounds__(256) void k_null_refine(KP k, cf *W1, const double2 *B, const unsigned int *mx,
                                                    const unsigned int *cnt, int64_t cap) {
    if ((int64_t)*cnt <= cap) return;
    const int r = blockIdx.y, lane = threadIdx.x & 63;
    const int64_t N = k.N, H = N / 2;
    const float band = fmaxf(1e-3f, 3e-5f * __uint_as_float(mx[r]));
    const int64_t nw = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);       // this wave's 64 samples
    const int64_t n = nw * 64 + lane;
    cf *z = W1 + (int64_t)r * k.N;
    uint64_t todo = __ballot(refine_cand(z, n, k.N, band));
    while (todo) {
        const int src = __ffsll((long long)todo) - 1;
        todo &= todo - 1;
        const int64_t ns = nw * 64 + src;
        const double m = refine_mask(k, B, r, ns, lane);
        if (lane == src) z[ns].y = m > 1.0 ? 2.0f : 0.0f;
    }
}

// ---------------------------------------------------------------------------
// odd N (utils.shift_t only): the reference's irfft without n= returns
// L = N - 1 samples -- the inverse of length L of the N-point spectrum's bins
// 0..M (M = (N - 1)/2), bin M taken as L's Nyquist bin (real part only):
//   y_m = (Re X_0 + 2 sum_{0<k<M} Re(X_k e^{2 pi i k m / L}) + Re X_M (-1)^m) / L
// with X = rfft(y) * ramp (utils.py:52-57).  Direct O(N^2) sums, f64
// accumulation, after the forward direct DFT (k_fb_dft<false>) into W2.
// ---------------------------------------------------------------------------
__global__ void k_odd_twiddles(cf *tw, int64_t L) {
    for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < L; m += (int64_t)gridDim.x * blockDim.x) {
        double s, c;
        sincospi(2.0 * (double)m / (double)L, &s, &c);
        tw[m] = make_float2((float)c, (float)s);
    }
}

__global__ __launch_bounds__(256) void k_odd_irfft(KP k, const cf *tw, float *rows, int64_t ld) {
    __shared__ cf tile[1024];
    const int r = blockIdx.y;
    const int64_t N = k.N, L = N - 1, M = L / 2;
    const cf *X = reinterpret_cast<const cf *>(k.p.work) + (int64_t)(k.p.nchan + r) * N;
    const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t mm = m < L ? m : 0;
    double acc = 0.0;
    for (int64_t base = 1; base < M; base += 1024) {
        const int cnt = (int)min((int64_t)1024, M - base);
        __syncthreads();
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) tile[i] = X[base + i];
        __syncthreads();
        int64_t j = (base * mm) % L;               // twiddle index (k m) mod L, advanced exactly
        for (int i = 0; i < cnt; ++i) {
            const cf w = tw[j], x = tile[i];
            acc += (double)x.x * w.x - (double)x.y * w.y;
            j += mm;
            if (j >= L) j -= L;
        }
    }
    if (m >= L) return;
    const double ends = (double)X[0].x + ((m & 1) ? -(double)X[M].x : (double)X[M].x);
    rows[(int64_t)r * ld + m] = (float)((ends + 2.0 * acc) / (double)L);
}

// ---------------------------------------------------------------------------
// path 3b: Bluestein (chirp-z) DFT for the fallback lengths N > 8192 (even N
// that are neither 2^m nor a mixed-radix split, e.g. the reference's own
// simulate fixture, 3 125 000 = 2^3 5^8; and delayed nulls on mixed-radix
// lengths).  With w_n = exp(-pi i n^2 / N) and nk = (n^2 + k^2 - (k-n)^2)/2:
//     X_k = w_k sum_n (x_n w_n) conj(w_{k-n}),
// a linear convolution evaluated as a circular one of length
// M = 2^ceil(log2(2N - 1)) through a power-of-two four-step M = M1 x M2
// (M2 = 4096, or 8192 for M = 2^25):
//     col pass  : a_n = x_n w_n (0 for n >= N), FFT over n1, twiddle  -> Z
//     row pass  : FFT over n2, * Bhat (same permuted order), inverse FFT
//     col pass  : conj twiddle, inverse FFT over k1, * w_k        -> X
// Bhat = FFT_M(b)/M, b_m = conj(w_m) for m < N, conj(w_{M-m}) for m > M - N,
// built by the same col/row kernels (mode 2).  The inverse DFT of the
// pipeline is conj(DFT(conj X)) / N through the same kernels; the forward
// DFT's last column pass and the inverse's first share one LDS block (KIND 2),
// so forward -> ramp -> inverse is 5 streaming passes over M complex per
// channel instead of the direct path's O(N^2); fp32 throughout (relative
// error ~2e-6 at M = 2^25).
// ---------------------------------------------------------------------------
struct BsArgs {
    const cf *src;     // mode 0/1: complex rows [nchan][N] (the W1 / W2 buffers)
    cf *dst;           // mode 0/1: complex rows [nchan][N]
    cf *Z;             // [nb][M] convolution workspace (mode 2: Bhat itself)
    const cf *chirp;   // [N]  w_n
    const cf *bhat;    // [M]  permuted order, scaled 1/M
    int64_t N, M, M1, M2;
    int64_t ld;        // row pitch of src / dst (complex): N, or N rounded up to a 128-B line
                       // for the fused pair runs' internal rows (rows of N = 2^20 - 2 would
                       // otherwise start 16 B off a line and split every segment in two)
    int r0;            // first channel (pair runs: pair) of this batch
    int fastio;        // fused first / last passes may take the one-sample-per-item
                       // forms on device-resident rows (0 under PSS_FLAG_NO_FAST)
    int mode;          // 0 forward DFT (+ delay ramp), 1 inverse DFT (/N), 2 Bhat build; pair runs:
                       // 3 inverse DFT's first pass (conj input), 4 forward DFT's last pass (X out)
};

// w_n = exp(-pi i n^2 / N): n^2 reduced mod 2N exactly, angle in double
__global__ void k_bs_chirp(cf *chirp, int64_t N) {
    for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < N;
         n += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t m = ((uint64_t)n * (uint64_t)n) % (uint64_t)(2 * N);
        double s, c;
        sincospi(-(double)m / (double)N, &s, &c);
        chirp[n] = make_float2((float)c, (float)s);
    }
}

// exp(sgn 2 pi i m / M), 0 <= m < M <= 2^25: |m| folded to <= M/2, exact in float
__device__ __forceinline__ cf bs_twiddle(int64_t m, int64_t M, float invM, bool inv) {
    const int64_t ms = (2 * m > M) ? m - M : m;
    const float r = (float)ms * invM;
    return expi_rev(inv ? r : -r);
}

template <int L, int B, int T, typename R>
struct BsFft;
template <int L, int B, int T, int... Rs>
struct BsFft<L, B, T, RList<Rs...>> {
    using FF = Fft<L, B, T>;
    // LDS (natural order, B sequences of L) -> transform -> LDS (natural)
    template <bool INV>
    __device__ static __forceinline__ void go(cf *lds, int tid) {
        cf v[FF::E];
        FF::template load<FF::template first<Rs...>()>(v, lds, tid);
        __syncthreads();                // the first stage's scatter rewrites LDS
        FF::template run<INV, 1, Rs...>(v, lds, tid);
        __syncthreads();
        FF::template store<FF::template last_of<Rs...>()>(v, lds, tid);
        __syncthreads();
    }
};

// Column pass over B = 8192 / L adjacent columns n2 (grid: M2 / B, batch rows).
// Column pass over B = 8192 / L adjacent columns n2 (grid: M2 / B, batch rows).
// KIND 0: first pass (a_n = src_n w_n, or b_m for the Bhat build) -> forward
// FFT -> twiddle -> Z.  KIND 2 (the middle of a forward + inverse DFT pair):
// conj twiddle -> inverse FFT -> X_n = conv_n w_n, delay ramp / transfer
// function, then the inverse DFT's input conj(X_n) w_n (0 for n >= N) ->
// forward FFT -> twiddle -> Z, all in one LDS block (no W2 round trip, one
// pass fewer).  KIND 1: last pass: conj twiddle -> inverse FFT -> conj(conv_n
// w_n) / N -> dst.
template <int L, typename R, int KIND>
__global__ __launch_bounds__(256) void k_bs_col(KP k, BsArgs a) {
    constexpr int B = 8192 / L, T = 256;
    __shared__ cf lds[B * Lds<L>::RS];
    const int tid = threadIdx.x, rb = blockIdx.y, r = a.r0 + rb;
    // XCD-aware block order: workgroup ids go round-robin over the 8 XCDs, so
    // blocks x, x + 8, ... (one XCD) take adjacent column ranges -- a 128-B
    // line a row offset splits between two neighbouring blocks (rows of N =
    // 2^20 - 2 complex start 16 B off a line) is fetched once into that
    // XCD's L2 instead of once per XCD
    const unsigned gx = gridDim.x;
    const unsigned bx = (gx & 7) ? blockIdx.x : (blockIdx.x & 7) * (gx >> 3) + (blockIdx.x >> 3);
    const int64_t n20 = (int64_t)bx * B;
    const float invM = 1.0f / (float)a.M;
    cf *Z = a.Z + (int64_t)rb * a.M;
    // NI items per thread; the first NH of them hold the rows n1 < M1 / 2,
    // i.e. n < M / 2: every sample n < N (M >= 2N) lies there, so the later
    // items are the zero padding (input) / discarded (output) at compile time
    constexpr int NI = L * B / T, NH = NI / 2;
    // loops unrolled (trip counts are compile-time): every load of a thread
    // in flight together (two 256-thread workgroups per CU leave few waves
    // to hide HBM latency otherwise)
    if constexpr (KIND == 3) {
        // pair runs, first pass with the source fused in: both channels of
        // pair r generated for 4 consecutive samples (one Philox block) per
        // item, (x_a + i x_b) w_n into the block (k_fb_source_pair's values)
        static_assert(B >= 4, "fused source: 4-sample items");
        const int ra = 2 * r - k.poff, rc = ra + 1;
        const bool hasa = ra >= 0, hasb = rc < k.p.nchan;
        if (a.fastio && k.p.src == PSS_SRC_LOAD && k.p.null_mode != PSS_NULL_UNDELAYED && hasa && hasb) {
            // rows already on the device (shift_t, filter_rows, disperse of a
            // made signal): no draws, so one sample per item with lanes along
            // the row (coalesced loads), every load issued before the first
            // is used; indices clamped, values zeroed arithmetically past N
            const float *rowa = k.p.data + (int64_t)ra * k.p.ld, *rowb = rowa + k.p.ld;
            float xa[NH], xb[NH];
            cf wv[NH];
#pragma unroll
            for (int it = 0; it < NH; ++it) {
                const int idx = tid + it * T;
                const int64_t n = (int64_t)(idx / B) * a.M2 + n20 + (idx & (B - 1));
                const int64_t nc = n < a.N ? n : 0;
                xa[it] = rowa[nc];
                xb[it] = rowb[nc];
                wv[it] = a.chirp[nc];
            }
#pragma unroll
            for (int it = 0; it < NI; ++it) {
                const int idx = tid + it * T;
                const int b = idx & (B - 1), n1 = idx / B;
                cf v = make_float2(0.f, 0.f);
                if (it < NH) {
                    const float f = (int64_t)n1 * a.M2 + n20 + b < a.N ? 1.0f : 0.0f;
                    v = cmul(make_float2(xa[it], xb[it]), wv[it]);
                    v = make_float2(v.x * f, v.y * f);
                }
                lds[Lds<L>::at(b, n1)] = v;
            }
        } else
#pragma unroll
        for (int it = 0; it < NI / 4; ++it) {
            const int idx = tid + it * T;
            const int b4 = (idx % (B / 4)) * 4, n1 = idx / (B / 4);
            const int64_t n = (int64_t)n1 * a.M2 + n20 + b4;
            float xa[4] = {0.f, 0.f, 0.f, 0.f}, xb[4] = {0.f, 0.f, 0.f, 0.f}, dum[4];
            const int cnt = (it < NH / 4 && n < a.N) ? (int)min((int64_t)4, a.N - n) : 0;
            if (cnt) {
                if (hasa) source4(k, ra, n, cnt, xa, dum, true, false);
                if (hasb) source4(k, rc, n, cnt, xb, dum, true, false);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
                lds[Lds<L>::at(b4 + i, n1)] = i < cnt ? cmul(make_float2(xa[i], xb[i]), a.chirp[n + i])
                                                     : make_float2(0.f, 0.f);
        }
    } else if (KIND == 0 && a.mode == 2) {
        // the Bhat build (one row, once per run): b_m = conj(w_m) for m < N,
        // conj(w_{M-m}) for m > M - N
#pragma unroll
        for (int it = 0; it < L * B / T; ++it) {
            const int idx = tid + it * T;
            const int b = idx & (B - 1), n1 = idx / B;
            const int64_t n = (int64_t)n1 * a.M2 + n20 + b;
            const int64_t m = n < a.N ? n : (n > a.M - a.N ? a.M - n : -1);
            lds[Lds<L>::at(b, n1)] = m >= 0 ? make_float2(a.chirp[m].x, -a.chirp[m].y) : make_float2(0.f, 0.f);
        }
    } else {
        // Every load of the block issued before the first value is used (two
        // 256-thread workgroups per CU: few waves to hide HBM latency).  As
        // one loop the compiler interleaved loads and LDS stores, 4 loads in
        // flight per wave; and a select around the first pass's loads became
        // a branch per item, each waiting on its own loads.
        constexpr int NL = KIND == 0 ? NH : NI;     // items loaded
        cf va[NL], vb[KIND == 0 ? NL : 1];
#pragma unroll
        for (int it = 0; it < NL; ++it) {
            const int idx = tid + it * T;
            const int b = idx & (B - 1), n1 = idx / B;
            const int64_t n = (int64_t)n1 * a.M2 + n20 + b;
            if (KIND == 0) {
                // a_n = x_n w_n (mode 3, pair runs' inverse DFT: conj(Y_n) w_n);
                // index clamped, the value zeroed arithmetically below
                const int64_t nc = n < a.N ? n : 0;
                va[it] = a.src[(int64_t)r * a.ld + nc];
                vb[it] = a.chirp[nc];
            } else {
                va[it] = Z[n];
            }
        }
#pragma unroll
        for (int it = 0; it < NI; ++it) {
            const int idx = tid + it * T;
            const int b = idx & (B - 1), n1 = idx / B;
            const int64_t n = (int64_t)n1 * a.M2 + n20 + b;
            cf v;
            if (KIND == 0) {
                if (it < NL) {
                    const float f = n < a.N ? 1.0f : 0.0f;
                    v = cmul(a.mode == 3 ? make_float2(va[it].x, -va[it].y) : va[it], vb[it]);
                    v = make_float2(v.x * f, v.y * f);
                } else {
                    v = make_float2(0.f, 0.f);
                }
            } else {
                // Q[k1 = n1][n2] * exp(+2 pi i n2 k1 / M)
                v = cmul(va[it], bs_twiddle((n20 + b) * n1, a.M, invM, true));
            }
            lds[Lds<L>::at(b, n1)] = v;
        }
    }
    __syncthreads();
    BsFft<L, B, T, R>::template go<KIND != 0 && KIND != 3>(lds, tid);
    if (KIND == 2) {
        int mtid = tid;                 // (opaque: see the output loop's otid)
        asm volatile("" : "+v"(mtid));
#pragma unroll
        for (int it = 0; it < L * B / T; ++it) {
            const int idx = mtid + it * T;
            const int b = idx & (B - 1), n1 = idx / B;
            const int64_t pos = (int64_t)n1 * a.M2 + n20 + b;
            cf v = make_float2(0.f, 0.f);
            if (it < NH && pos < a.N) {
                const cf w = a.chirp[pos];
                const cf X = apply_ramp(k, r, pos, cmul(lds[Lds<L>::at(b, n1)], w));
                v = cmul(make_float2(X.x, -X.y), w);
            }
            lds[Lds<L>::at(b, n1)] = v;
        }
        __syncthreads();
        BsFft<L, B, T, R>::template go<false>(lds, tid);
    }
    const float invN = 1.0f / (float)a.N;
    // the output loop's indices and twiddles from an opaque copy of the
    // thread id: computed here, not hoisted above the FFT and held through it
    // (that had KIND 0 at 294 VGPRs, one wave per SIMD)
    int otid = tid;
    asm volatile("" : "+v"(otid));
    // KIND 1 / 4: the chirp at this thread's output positions, all loaded
    // before the first is used (as a load inside the output loop each item's
    // store waited on its own load; loaded with the input instead, the
    // values held through the FFT pushed the kernel past 256 VGPRs)
    cf cw[(KIND == 1 || KIND == 4) ? NH : 1];
    if constexpr (KIND == 1 || KIND == 4) {
#pragma unroll
        for (int it = 0; it < NH; ++it) {
            int64_t pos;
            if constexpr (KIND == 1) {          // the output loop's items
                const int idx = otid + it * T;
                pos = (int64_t)(idx / B) * a.M2 + n20 + (idx & (B - 1));
            } else {                            // 4-sample items: it = 4 item + i
                const int idx = otid + (it >> 2) * T;
                pos = (int64_t)(idx / (B / 4)) * a.M2 + n20 + (idx % (B / 4)) * 4 + (it & 3);
            }
            cw[it] = a.chirp[pos < a.N ? pos : 0];
        }
    }
    if constexpr (KIND == 4) {
        // pair runs, last pass with the epilogue fused in: y = conj(conv_n
        // w_n) / N = (y_a + i y_b) of 4 consecutive samples per item, each
        // channel's epilogue (null replacement, observe copy, noise, store)
        // straight from the block (k_fb_epilogue_pair's values)
        static_assert(B >= 4, "fused epilogue: 4-sample items");
        const int ra = 2 * r - k.poff, rc = ra + 1;
        const bool hasa = ra >= 0, hasb = rc < k.p.nchan;
        if (a.fastio && !k.p.noise && k.p.null_mode != PSS_NULL_DELAYED && k.p.out_kind == PSS_OUT_NONE && hasa &&
            hasb) {
            // the epilogue is a plain store (shift_t, filter_rows, disperse
            // of a made signal): one sample per item, lanes along the row
            // (coalesced stores), the chirp of the NH items loaded as a batch
            float *oa = k.p.data + (int64_t)ra * k.p.ld, *ob = oa + k.p.ld;
            cf c1[NH];
#pragma unroll
            for (int it = 0; it < NH; ++it) {
                const int idx = otid + it * T;
                const int64_t pos = (int64_t)(idx / B) * a.M2 + n20 + (idx & (B - 1));
                c1[it] = a.chirp[pos < a.N ? pos : 0];
            }
#pragma unroll
            for (int it = 0; it < NH; ++it) {
                const int idx = otid + it * T;
                const int b = idx & (B - 1), k1 = idx / B;
                const int64_t pos = (int64_t)k1 * a.M2 + n20 + b;
                if (pos < a.N) {
                    const cf v = cmul(lds[Lds<L>::at(b, k1)], c1[it]);
                    oa[pos] = v.x * invN;
                    ob[pos] = -v.y * invN;
                }
            }
            return;
        }
        const float msk[4] = {0.f, 0.f, 0.f, 0.f};
        // y = conj(conv w) / N back into the thread's own LDS entries first
        // (a small loop, unrolled: cw stays in registers; the epilogue loop
        // below is too large to unroll, and indexing cw there put it in scratch)
#pragma unroll
        for (int it = 0; it < NH / 4; ++it) {
            const int idx = otid + it * T;
            const int b4 = (idx % (B / 4)) * 4, k1 = idx / (B / 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const cf v = cmul(lds[Lds<L>::at(b4 + i, k1)], cw[4 * it + i]);
                lds[Lds<L>::at(b4 + i, k1)] = make_float2(v.x * invN, -v.y * invN);
            }
        }
        for (int it = 0; it < NH / 4; ++it) {
            const int idx = otid + it * T;
            const int b4 = (idx % (B / 4)) * 4, k1 = idx / (B / 4);
            const int64_t pos = (int64_t)k1 * a.M2 + n20 + b4;
            if (pos >= a.N) continue;
            const int cnt = (int)min((int64_t)4, a.N - pos);
            float ya[4] = {0.f, 0.f, 0.f, 0.f}, yb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (i < cnt) {
                    const cf v = lds[Lds<L>::at(b4 + i, k1)];
                    ya[i] = v.x;
                    yb[i] = v.y;
                }
            }
            if (hasa) epilogue4(k, ra, pos, cnt, ya, msk, false);
            if (hasb) epilogue4(k, rc, pos, cnt, yb, msk, false);
        }
        return;
    }
#pragma unroll
    for (int it = 0; it < (KIND == 1 ? NH : NI); ++it) {
        const int idx = otid + it * T;
        const int b = idx & (B - 1), k1 = idx / B;
        const int64_t n2 = n20 + b, pos = (int64_t)k1 * a.M2 + n2;
        cf v = lds[Lds<L>::at(b, k1)];
        if (KIND != 1) {
            Z[pos] = cmul(v, bs_twiddle(n2 * k1, a.M, invM, false));
        } else if (pos < a.N) {                 // pos = n1 M2 + n2: output sample
            v = cmul(v, cw[KIND == 1 ? it : 0]);
            // mode 4 (pair runs: the forward DFT's last pass): X_n, unscaled
            a.dst[(int64_t)r * a.ld + pos] = a.mode == 4 ? v : make_float2(v.x * invN, -v.y * invN);
        }
    }
}

// Pair runs (no delayed null: two real channels per complex Bluestein row,
// half the transforms).  Between the forward DFT (X, natural order, in W1)
// and the inverse: per pair row and bin k <= N/2, the two channels'
// spectra A = (X_k + conj X_{N-k}) / 2, B = (X_k - conj X_{N-k}) / 2i, each
// times its own channel's ramp / transfer function (apply_ramp: A and B are
// real at DC and Nyquist, so the real-part rule applies), recombined as
// Y_k = A' + i B', Y_{N-k} = conj A' + i conj B'.  In place; rows of the
// batch starting at pair r0 (local channel rows 2 p - poff, 2 p + 1 - poff).
__global__ __launch_bounds__(256) void k_bs_sep(KP k, cf *X, int64_t ld, int r0) {
    const int p = r0 + (int)blockIdx.y;
    const int ra = 2 * p - k.poff, rb = ra + 1;
    const int ca = max(ra, 0), cb = min(rb, k.p.nchan - 1);
    const int64_t N = k.N, H = N / 2;
    cf *x = X + (int64_t)p * ld;
    for (int64_t kb = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; kb <= H;
         kb += (int64_t)gridDim.x * blockDim.x) {
        const int64_t km = kb ? N - kb : 0;
        const cf z = x[kb], zm = x[km];
        cf A = make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
        cf B = make_float2(0.5f * (z.y + zm.y), 0.5f * (zm.x - z.x));
        if (kb == 0 || kb == H) {                     // real bins (rounding residue dropped)
            A.y = 0.0f;
            B.y = 0.0f;
        }
        A = apply_ramp(k, ca, kb, A);
        B = apply_ramp(k, cb, kb, B);
        x[kb] = make_float2(A.x - B.y, A.y + B.x);
        if (kb != km) x[km] = make_float2(A.x + B.y, B.x - A.y);
    }
}

// Pair runs: source of both channels of a pair into one complex row, and the
// epilogue of both from it (the k_fb_source / k_fb_epilogue of the channel rows).
__global__ __launch_bounds__(256) void k_fb_source_pair(KP k) {
    const int p = blockIdx.y;
    const int ra = 2 * p - k.poff, rb = ra + 1;
    const bool hasa = ra >= 0, hasb = rb < k.p.nchan;
    cf *W1 = reinterpret_cast<cf *>(k.p.work) + (int64_t)p * k.N;
    const int64_t items = (k.N + 3) >> 2;
    for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < items;
         it += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n0 = it << 2;
        const int cnt = (int)min((int64_t)4, k.N - n0);
        float a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0}, dum[4];
        if (hasa) source4(k, ra, n0, cnt, a, dum, true, false);
        if (hasb) source4(k, rb, n0, cnt, b, dum, true, false);
        for (int i = 0; i < cnt; ++i) W1[n0 + i] = make_float2(a[i], b[i]);
    }
}
__global__ __launch_bounds__(256) void k_fb_epilogue_pair(KP k) {
    const int p = blockIdx.y;
    const int ra = 2 * p - k.poff, rb = ra + 1;
    const bool hasa = ra >= 0, hasb = rb < k.p.nchan;
    const cf *W1 = reinterpret_cast<const cf *>(k.p.work) + (int64_t)p * k.N;
    const int64_t items = (k.N + 3) >> 2;
    for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < items;
         it += (int64_t)gridDim.x * blockDim.x) {
        const int64_t n0 = it << 2;
        const int cnt = (int)min((int64_t)4, k.N - n0);
        float a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
        const float msk[4] = {0, 0, 0, 0};
        for (int i = 0; i < cnt; ++i) {
            const cf z = W1[n0 + i];
            a[i] = z.x;
            b[i] = z.y;
        }
        if (hasa) epilogue4(k, ra, n0, cnt, a, msk, false);
        if (hasb) epilogue4(k, rb, n0, cnt, b, msk, false);
    }
}

// Row pass over one row k1 of M2 (grid: M1, batch rows): forward FFT, then
// mode 2: scale 1/M and store (Bhat); else * Bhat, inverse FFT, store.
template <int L, typename F, typename I>
struct BsRow;
template <int L, int... F, int... I>
struct BsRow<L, RList<F...>, RList<I...>> {
    static constexpr int T = L / 16;
    using FF = Fft<L, 1, T>;
    __device__ static void go(const KP &k, const BsArgs &a) {
        (void)k;
        __shared__ cf lds[Lds<L>::RS];
        const int tid = threadIdx.x, k1 = blockIdx.x;
        cf *row = a.Z + (int64_t)blockIdx.y * a.M + (int64_t)k1 * L;
#pragma unroll
        for (int i = 0; i < L / T; ++i) lds[Lds<L>::at(0, tid + i * T)] = row[tid + i * T];
        __syncthreads();
        cf v[FF::E];
        FF::template load<FF::template first<F...>()>(v, lds, tid);
        __syncthreads();
        FF::template run<false, 1, F...>(v, lds, tid);
        constexpr int RFL = FF::template last_of<F...>();
        constexpr int RIL = FF::template last_of<I...>();
        if (a.mode == 2) {
            const float invM = 1.0f / (float)a.M;
#pragma unroll
            for (int i = 0; i < FF::E; ++i) {
                int b, pos;
                FF::template where<RFL>(i, tid, b, pos);
                row[pos] = make_float2(v[i].x * invM, v[i].y * invM);
            }
            return;
        }
        const cf *bh = a.bhat + (int64_t)k1 * L;
#pragma unroll
        for (int i = 0; i < FF::E; ++i) {
            int b, pos;
            FF::template where<RFL>(i, tid, b, pos);
            v[i] = cmul(v[i], bh[pos]);
        }
        FF::template run<true, 1, I...>(v, lds, tid);
#pragma unroll
        for (int i = 0; i < FF::E; ++i) {
            int b, pos;
            FF::template where<RIL>(i, tid, b, pos);
            row[pos] = v[i];
        }
    }
};

template <typename RW>
__global__ __launch_bounds__(RW::T) void k_bs_row(KP k, BsArgs a) {
    RW::go(k, a);
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
            const float f = fminf(fmaxf((float)v, -128.f), 127.f);
            ((int8_t *)out)[e] = (int8_t)(int)truncf(f);
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

// ---------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------
static inline bool is_pow2(int64_t n) { return n > 0 && (n & (n - 1)) == 0; }

static dim3 stream_grid(int64_t items, int rows) {
    int64_t bx = (items + 255) / 256;
    if (bx > 4096) bx = 4096;
    if (bx < 1) bx = 1;
    return dim3((unsigned)bx, (unsigned)rows, 1);
}


template <int L, int BATCH, int T, typename F, typename I>
static int launch_single(const KP &k, hipStream_t st) {
    using SP = SinglePass<L, BATCH, T, F, I>;
    dim3 grid((k.p.nchan + BATCH - 1) / BATCH);
    tk_begin(TK_SINGLE, st);
    k_single<SP, T><<<grid, dim3(T), 0, st>>>(k);
    tk_end(st);
    LAUNCHCHK();
    return PSS_OK;
}

// Column plans: B*N1 = 8192 complex per workgroup, 512 threads, 16 per thread.
// Inverse plans (..I) mirror the forward ones where registers carry over
// (single pass, rows); column inverses start from LDS and reuse the forward plan.
// Row plans: N2 = 8192 (1 row, 512 thr) or N2 <= 4096 (4096/N2 rows, 256 thr).
using C16 = RList<16>;
using C32F = RList<16, 2>;
using C32I = RList<2, 16>;
using C64F = RList<16, 4>;
using C64I = RList<4, 16>;
using C128F = RList<16, 8>;
using C128I = RList<8, 16>;
using C256 = RList<16, 16>;
using C512F = RList<16, 16, 2>;
using C512I = RList<2, 16, 16>;
using C1kF = RList<16, 16, 4>;
using C1kI = RList<4, 16, 16>;
using C2kF = RList<16, 16, 8>;
using C2kI = RList<8, 16, 16>;
using C4k = RList<16, 16, 16>;
using C8kF = RList<16, 8, 8, 8>;
using C8kI = RList<8, 8, 8, 16>;
using C16kF = RList<16, 16, 8, 8>;
using C16kI = RList<8, 8, 16, 16>;

// ---------------------------------------------------------------------------
// workspace layout (every region 256-B aligned)
//   four-step (N = 2^m, 2^14 <= N <= 2^24):
//     Yd [npairs][N] cf | Mspec [N] cf | node spill [KCH/2][N] cf |
//     nodes [KCH][N] f32 | table bits [N/64] uint4 | base [N/64] u32 |
//     coef [N][KREC] f32 (worst case) | misc (counter, node ramps/nyq) |
//     null bits [nchan][N/32] u32 | mask row [N] f32
//   single pass (N <= 8192): mask row
//   direct DFT fallback: W1, W2 [nchan][N] cf | twiddles [N] cf | mask row
// ---------------------------------------------------------------------------
static inline int64_t al256(int64_t b) { return (b + 255) & ~255ll; }
static inline bool fourstep_len(int64_t n) { return is_pow2(n) && n >= 16384 && n <= (1ll << 24); }

// Mixed-radix four-step lengths: even N = N1 * N2 with N2 = 2^m in
// [1024, 8192] (the largest such power that leaves N1 even) and N1 one of the
// {2, 3, 4, 5}-smooth column lengths below (e.g. the fold-mode C4 length
// 30720 = 30 x 1024).  Other even lengths take the direct path.
static inline bool smooth_col(int64_t n1) {
    switch (n1) {
        case 6: case 10: case 12: case 20: case 24: case 30: case 40: case 48: case 60: return true;
        default: return false;
    }
}
// 5-smooth lengths with few factors of two take an LDS four-step with
// radix-5 stages both ways: 3 125 000 = 2^3 5^8 (the sample count of the
// reference's own simulate fixture, tests/test_simulate.py:47-56) as 1250
// columns (2 x 5^4) x rows of 2500 (4 x 5^4).
static inline bool smooth5_split(int64_t n, int64_t *N1 = nullptr, int64_t *N2 = nullptr) {
    if (n != 3125000) return false;
    if (N1) *N1 = 1250;
    if (N2) *N2 = 2500;
    return true;
}
static inline bool smooth_split(int64_t n, int64_t *N1 = nullptr, int64_t *N2 = nullptr) {
    if (smooth5_split(n, N1, N2)) return true;
    if (n <= 0 || (n & 1) || is_pow2(n) || n > (1ll << 24)) return false;
    int v2 = __builtin_ctzll((unsigned long long)n);
    const int m = v2 - 1 < 13 ? v2 - 1 : 13;            // keep N1 even
    if (m < 10) return false;
    const int64_t n2 = 1ll << m, n1 = n / n2;
    if (!smooth_col(n1)) return false;
    if (N1) *N1 = n1;
    if (N2) *N2 = n2;
    return true;
}

static int g_flags = 0;   // pss_set_flags (test hook)

// Bluestein geometry of a fallback length N > 8192 (path 3b): M = M1 x M2,
// nb channels per convolution batch (the batch buffer is about one W buffer).
struct BsGeom { int64_t M, M1, M2, nb; };
static inline bool bs_len(int64_t N) { return N > 8192 && N <= (1ll << 24); }
static BsGeom bs_geom(int32_t nchan, int64_t N) {
    BsGeom g;
    g.M = 1;
    while (g.M < 2 * N - 1) g.M <<= 1;
    g.M2 = g.M >= (1ll << 25) ? 8192 : 4096;
    g.M1 = g.M / g.M2;
    g.nb = ((int64_t)nchan * N + g.M - 1) / g.M;    // (ceil: no near-empty last batch)
    if (g.nb < 1) g.nb = 1;
    if (g.nb > nchan) g.nb = nchan;
    if (g.nb > 65535) g.nb = 65535;
    return g;
}

struct WsLayout {
    int64_t yd, mspec, ynode, nodes, bits, base, coef, misc, mbits, rtab, wlist, row, total;
    int64_t bs_chirp, bs_bhat, bs_z;   // Bluestein: w [N] | Bhat [M] | Z [nb][M] (cf)
    int64_t odd_tw;                    // odd N: exp(+2 pi i j / (N - 1)), j < N - 1 (cf)
    int64_t rf_tw, rf_B, rf_mx;        // float64 null decisions: e^{2 pi i n/N} [N], B [N/2+1] (double2), row max [nchan]
    int64_t rf_part, rf_list, rf_cnt;  // ... partial spectra [kBsParts][N/2+1] (double2), candidate list, its count
};

static WsLayout ws_layout(int32_t nchan, int64_t N, bool filt = false) {
    WsLayout w;
    memset(&w, 0, sizeof(w));
    int64_t o = 0;
    if (fourstep_len(N)) {
        const int64_t npairs = ((int64_t)nchan + 2) / 2;   // pairs of (even, odd) global channels
        // pair spills: N1 x N2 complex per pair
        const int64_t ps = N;
        w.yd = o;    o += al256(npairs * ps * 8);
        w.mspec = o; o += al256(N * 8);
        w.ynode = o; o += al256((int64_t)(KCH / 2) * ps * 8);
        w.nodes = o; o += al256((int64_t)KCH * N * 4);
        w.bits = o;  o += al256((N / 32) * 8);
        w.base = o;  o += al256((N / 32) * 4);
        w.coef = o;  o += al256(N * KREC * 4);
        w.misc = o;  o += 256;
        w.mbits = o; o += al256((int64_t)nchan * (N / 8));   // per-channel null bits
        w.rtab = o;  o += al256(npairs * 2 * 64 * 8);          // row-pass pair ramp factors (RFL <= 64)
        w.wlist = o; o += al256((N / 32) * 4);                 // null fix-up: table words with nulls
    } else if (filt || !(is_pow2(N) && N >= 64 && N <= 8192)) {
        // fallback: W1, W2, twiddles -- Bluestein needs W1 only (its forward
        // and inverse DFTs are fused through Z), unless the mixed-radix
        // four-step shares these bytes or the direct DFT is forced
        const bool odd = (N & 1) != 0;
        const bool w1_only = bs_len(N) && !odd && !smooth_split(N) && !(g_flags & PSS_FLAG_DIRECT_DFT);
        o += al256(w1_only ? (int64_t)nchan * N * 8 : 2 * (int64_t)nchan * N * 8 + N * 8);
        if (odd) {
            // odd-length shift_t: twiddles of the (N - 1)-point inverse
            w.odd_tw = o;
            o += al256((N - 1) * 8);
        } else if (bs_len(N)) {
            const BsGeom g = bs_geom(nchan, N);
            w.bs_chirp = o; o += al256(N * 8);
            w.bs_bhat = o;  o += al256(g.M * 8);
            w.bs_z = o;     o += al256(g.nb * g.M * 8);
        }
        if (!odd && N <= kRefineMaxN) {
            w.rf_tw = o; o += al256(N * 16);
            w.rf_B = o;  o += al256((N / 2 + 1) * 16);
            w.rf_mx = o; o += al256((int64_t)nchan * 4);
            w.rf_part = o; o += al256((int64_t)kBsParts * (N / 2 + 1) * 16);
            w.rf_list = o; o += al256(refine_cap(nchan, N) * 8);
            w.rf_cnt = o;  o += 256;
        }
        if (smooth_split(N)) {
            // mixed-radix four-step (inside the same bytes: the direct path
            // still serves these lengths for a delayed null)
            const int64_t npairs = ((int64_t)nchan + 2) / 2;
            w.yd = 0;
            w.rtab = al256(npairs * N * 8);
        }
    }
    w.row = o;
    o += al256(N * 4);
    w.total = o;
    return w;
}

// Fast-path selection (kernels specialised for the north-star configuration;
// results are bitwise identical to the generic kernels).

static bool fast_source(const PssPipeline &p) {
    if (g_flags & PSS_FLAG_NO_FAST) return false;
    // (nint == knot_m: the table spans the period, so the fast walk needs no
    // extrapolation clamp -- pulsar._device_table always builds it so)
    return p.src == PSS_SRC_SEARCH && !p.gen_amp && p.gen_df == 1.0f && !p.inj_gen && p.null_mode != PSS_NULL_UNDELAYED &&
           p.nint <= kFastNint && !p.prof_split && (uint32_t)p.nint == p.knot_m;
}
// Fold-mode fast passes of the mixed-radix split (PairCols::passA_fold /
// passC_fold): the fold source with chi2(df != 1) pair draws, and an
// epilogue of noise only (any df != 1), no injected draws.
static bool fold_source(const PssPipeline &p) {
    if (g_flags & PSS_FLAG_NO_FAST) return false;
    return p.src == PSS_SRC_FOLD && !p.gen_amp && !p.inj_gen && p.gen_df != 1.0f && p.nph > 0 &&
           p.null_mode != PSS_NULL_UNDELAYED;
}
static bool fold_epilogue(const KP &k) {
    const PssPipeline &p = k.p;
    if (g_flags & PSS_FLAG_NO_FAST) return false;
    if (p.out_kind != PSS_OUT_NONE || p.inj_noise || p.inj_rep) return false;
    return p.noise && p.noise_df != 1.0f && p.null_mode != PSS_NULL_DELAYED;
}
static bool fast_epilogue(const KP &k) {
    const PssPipeline &p = k.p;
    if (g_flags & PSS_FLAG_NO_FAST) return false;
    if (p.out_kind != PSS_OUT_NONE || p.inj_noise || p.inj_rep) return false;
    if (!p.noise || p.noise_df != 1.0f) return false;
    if (p.null_mode == PSS_NULL_UNDELAYED) return false;
    if (p.null_mode == PSS_NULL_DELAYED && (!k.mtab || p.null_rep_df != 1.0f)) return false;
    return (p.ld % 4) == 0 && (((uintptr_t)p.data) & 15) == 0;
}

// Mask table of a delayed null (see the comment above KCH): mask spectrum,
// KCH node shifts (KCH/2 pair rows through the row and column engines),
// Chebyshev coefficients + classification.  Once per run, channel independent.
template <int N1, int B, int T, typename CF, typename CI, int N2, int TR, typename RF, typename RI,
          int TRF>
static int build_mask_table(KP &k, hipStream_t st, const float *mask_row, char *w, const WsLayout &L) {
    using PC = PairCols<N1, B, T, CF, CI>;
    using PR = PairRows<N2, TR, RF, RI>;
    cf *mspec = reinterpret_cast<cf *>(w + L.mspec);
    uint32_t *counter = reinterpret_cast<uint32_t *>(w + L.misc);
    uint64_t *nramp = reinterpret_cast<uint64_t *>(w + L.misc + 64);
    float *nnyq = reinterpret_cast<float *>(w + L.misc + 192);
    float *nodes = reinterpret_cast<float *>(w + L.nodes);
    int log2n = 0;
    while ((1ll << log2n) < k.N) ++log2n;
    // spectrum of the (channel independent) mask row
    KP km = k;
    km.p.nchan = 1;
    km.p.chan0 = 0;
    km.p.data = const_cast<float *>(mask_row);
    km.p.ld = k.N;
    km.p.src = PSS_SRC_LOAD;
    km.p.null_mode = PSS_NULL_NONE;
    km.p.data_in_fft = 1;
    km.p.work = mspec;
    using C1 = Cols<N1, B, T, CF, CI>;
    using R1 = Rows<N2, 1, TRF, RF, RI, true>;
    k_colA<C1, T><<<dim3((unsigned)(N2 / B), 1), dim3(T), 0, st>>>(km);
    LAUNCHCHK();
    k_row<R1, TRF><<<dim3((unsigned)N1, 1), dim3(TRF), 0, st>>>(km);
    LAUNCHCHK();
    // node shifts
    k_node_params<<<1, 64, 0, st>>>(nramp, nnyq, log2n);
    LAUNCHCHK();
    KP kn = k;
    kn.p.nchan = KCH;
    kn.p.chan0 = 0;
    kn.p.ramp = nramp;
    kn.p.nyq_re = nnyq;
    kn.p.nyq_im = nnyq;
    kn.poff = 0;
    kn.npairs = KCH / 2;
    kn.Ym = reinterpret_cast<cf *>(w + L.ynode);
    kn.Mspec = mspec;
    k_node_row<PR, TR><<<dim3((unsigned)(KCH / 2), (unsigned)(N1 / 2)), dim3(TR), 0, st>>>(kn);
    LAUNCHCHK();
    k_node_col<PC, T><<<dim3((unsigned)(N2 / B), (unsigned)(KCH / 2)), dim3(T), 0, st>>>(kn, nodes);
    LAUNCHCHK();
    // table
    HIPCHK(hipMemsetAsync(counter, 0, 4, st));
    k.mt_bits = reinterpret_cast<const uint2 *>(w + L.bits);
    k.mt_base = reinterpret_cast<const uint32_t *>(w + L.base);
    k.mt_coef = reinterpret_cast<const float *>(w + L.coef);
    k_mask_table<<<dim3((unsigned)(k.N / 256)), dim3(256), 0, st>>>(
        nodes, k.N, reinterpret_cast<uint2 *>(w + L.bits), reinterpret_cast<uint32_t *>(w + L.base),
        reinterpret_cast<float *>(w + L.coef), counter);
    LAUNCHCHK();
    {
        uint32_t *wl = reinterpret_cast<uint32_t *>(w + L.wlist);
        uint32_t *wcount = reinterpret_cast<uint32_t *>(w + L.misc + 8);
        HIPCHK(hipMemsetAsync(wcount, 0, 4, st));
        const uint32_t nwords = (uint32_t)(k.N / 32);
        k_mask_words<<<dim3((nwords + 255) / 256), dim3(256), 0, st>>>(k.mt_bits, nwords, wl, wcount);
        LAUNCHCHK();
        k.wlist = wl;
        k.nwlist = wcount;
    }
    k.mtab = 1;
    k.log2n = log2n;
    if (k.p.data_in_fft && !fast_epilogue(k)) {   // generic pass C reads the decisions as bits
        k.mbB = B;
        uint32_t *bm = reinterpret_cast<uint32_t *>(w + L.mbits);
        k_mask_bits<<<dim3((unsigned)((k.N / 32 + 255) / 256), (unsigned)k.p.nchan), dim3(256), 0, st>>>(k, bm);
        LAUNCHCHK();
        k.mbits = bm;
    }
    return PSS_OK;
}

// Extra LDS row pitch of the column kernels (tools/lds_banks.py): pass A's
// spill-store loop reads 4 columns x 16 rows per 32-lane group (a 32/B pitch
// offset spreads the columns over the 64 read banks); pass C's load loop
// writes 4 columns x 4 rows per 16-lane group (16/B over the 32 write banks).
// B < 32: a pitch that is a multiple of 16 complex, so the wave-local column
// FFTs get the byte-address exchanges (Fft::XB: round 2's 4-complex pad cost
// ~100 address VALU per lane in pass A); the spill-store loop then reads 32
// consecutive rows of one 4-column group per 32-lane group (conflict-free at
// any pitch, passA).
constexpr int xrs_read(int B) { return B >= 32 ? 1 : 16; }
// (pass C measured 0.5 ms faster on the padded layout at C3: its transposes
// gain nothing from the swizzle and the XOR addressing costs VALU)
constexpr int xrs_write(int B) { return -1; }

struct SideStreams {
    hipStream_t s[2];
    hipEvent_t ev[40];
    bool ok;
};
static SideStreams *side_streams() {
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

template <int N1, int B, int T, typename CF, typename CI, int N2, int TR, typename RF, typename RI,
          int TRF, int BC, int TC>
static int launch_pair_passes(KP &k, hipStream_t st);

// BC/TC: column-block width and threads of the FAST pass C (the spill layout
// does not depend on the block width, so pass C may use wider blocks than pass
// A: its output rows are written in BC-sample (4 BC-byte) segments).
template <int N1, int B, int T, typename CF, typename CI, int N2, int TR, typename RF, typename RI,
          int TRF, int BC = B, int TC = T>
static int launch_pair(KP &k, hipStream_t st, const float *mask_row) {
    using PC = PairCols<N1, B, T, CF, CI, xrs_read(B)>;
    using PCC = PairCols<N1, BC, TC, CF, CI, xrs_write(BC)>;
    using PR = PairRows<N2, TR, RF, RI>;
    k.poff = k.p.chan0 & 1;
    k.npairs = (k.p.nchan + k.poff + 1) / 2;
    char *w = reinterpret_cast<char *>(k.p.work);
    const WsLayout L = ws_layout(k.p.nchan, k.N);
    k.Yd = reinterpret_cast<cf *>(w + L.yd);
    if (k.p.null_mode == PSS_NULL_DELAYED) {
        // the mask table's position arithmetic is for N = 2^m (validate()
        // sends delayed nulls of other lengths to the direct path)
        if constexpr ((N1 & (N1 - 1)) == 0 && N2 <= 8192) {
            // With the data in the FFT and the fast passes, nothing reads the
            // table before the null fix-up: build it on a side stream next to
            // pass A (its dozen small launches then cost no time on the main
            // stream); the fix-up waits for it.
            SideStreams *ss = k.p.data_in_fft ? side_streams() : nullptr;
            hipStream_t ms = st;
            if (ss) {
                HIPCHK(hipEventRecord(ss->ev[30], st));
                HIPCHK(hipStreamWaitEvent(ss->s[0], ss->ev[30], 0));
                ms = ss->s[0];
            }
            const int rc = build_mask_table<N1, B, T, CF, CI, N2, TR, RF, RI, TRF>(k, ms, mask_row, w, L);
            if (rc) return rc;
            if (ss) {
                HIPCHK(hipEventRecord(ss->ev[31], ms));
                k.mask_ready = ss->ev[31];
            }
        } else {
            return fail(PSS_EUNSUPPORTED, "delayed null on the mixed-radix or 16384-row four-step (N=%lld)",
                        (long long)k.N);
        }
    }
    if (!k.p.data_in_fft) {
        // only the null mask was delayed: one elementwise pass with table lookups
        dim3 g = stream_grid((k.N + 3) / 4, k.p.nchan);
        tk_begin(TK_ELEM, st);
        k_elementwise<<<g, dim3(256), 0, st>>>(k);
        tk_end(st);
        LAUNCHCHK();
        return PSS_OK;
    }
    if (!k.p.htab) {   // (a transfer-function run has no ramps)
        cf *rt = reinterpret_cast<cf *>(w + L.rtab);
        k_pair_tab<PR::RFL><<<dim3((unsigned)k.npairs), dim3(64), 0, st>>>(k.p.ramp, k.N, k.p.nchan, k.poff,
                                                                          k.npairs, rt);
        LAUNCHCHK();
        k.rtab = rt;
    }
    return launch_pair_passes<N1, B, T, CF, CI, N2, TR, RF, RI, TRF, BC, TC>(k, st);
}

// The passes of one pair range (after the mask table and the ramp table).
template <int N1, int B, int T, typename CF, typename CI, int N2, int TR, typename RF, typename RI,
          int TRF, int BC, int TC>
static int launch_pair_passes(KP &k, hipStream_t st) {
    using PC = PairCols<N1, B, T, CF, CI, xrs_read(B)>;
    using PCC = PairCols<N1, BC, TC, CF, CI, xrs_write(BC)>;
    using PR = PairRows<N2, TR, RF, RI>;
    dim3 gc((unsigned)(N2 / B), (unsigned)k.npairs);
    tk_begin(TK_COLA, st);
    bool launched = false;
    if constexpr (PC::kRegCols) {
        if (fold_source(k.p)) {
            k_pairA_fold<PC, T><<<gc, dim3(T), 0, st>>>(k);
            launched = true;
        }
    }
    if (launched) {
    } else if constexpr (PC::kItemsExact) {
        if (fast_source(k.p)) {
            if (k.p.prof_rows == 1) k_pairA_fast<PC, T, true><<<gc, dim3(T), 0, st>>>(k);
            else k_pairA_fast<PC, T, false><<<gc, dim3(T), 0, st>>>(k);
        } else {
            k_pairA<PC, T><<<gc, dim3(T), 0, st>>>(k);
        }
    } else {
        k_pairA<PC, T><<<gc, dim3(T), 0, st>>>(k);
    }
    tk_end(st);
    LAUNCHCHK();
    tk_begin(TK_ROW, st);
    if constexpr (N2 > 8192) {
        // 16384-point rows (C5's 1024 x 16384 split): one row at a time
        // (PairRowsSeq); no transfer function / tail variant (run_fourstep
        // keeps those runs on the 2048 x 8192 split)
        if (k.p.htab || k.p.tail_a) return fail(PSS_EUNSUPPORTED, "%d-point rows: no transfer function", N2);
        // (16 values of each row per thread: 512 threads with 32 measured
        // 47.8 against 43.9 ms at C5, profiles/r05/r16/)
        constexpr int TS = N2 / 16;
        using PRS = PairRowsSeq<N2, TS, RF, RI>;
        k_pair_row_seq<PRS, TS, false><<<dim3((unsigned)k.npairs, (unsigned)(N1 / 2 - 1)), dim3(TS), 0, st>>>(k);
        k_pair_row_seq<PRS, TS, true><<<dim3((unsigned)k.npairs, 1u), dim3(TS), 0, st>>>(k);
    } else if (k.p.htab) {
        k_pair_row<PR, TR, false, true><<<dim3((unsigned)k.npairs, (unsigned)(N1 / 2)), dim3(TR), 0, st>>>(k);
    } else if (k.p.tail_a) {
        k_pair_row<PR, TR, true><<<dim3((unsigned)k.npairs, (unsigned)(N1 / 2)), dim3(TR), 0, st>>>(k);
    } else if constexpr (N2 == 8192) {
        constexpr int TS = N2 / 16;                  // 16 values of each row per thread
        using PRS = PairRowsSeq<N2, TS, RF, RI>;
        k_pair_row_seq<PRS, TS, false><<<dim3((unsigned)k.npairs, (unsigned)(N1 / 2 - 1)), dim3(TS), 0, st>>>(k);
        k_pair_row_seq<PRS, TS, true><<<dim3((unsigned)k.npairs, 1u), dim3(TS), 0, st>>>(k);
    } else {
        k_pair_row<PR, TR><<<dim3((unsigned)k.npairs, (unsigned)(N1 / 2)), dim3(TR), 0, st>>>(k);
    }
    tk_end(st);
    LAUNCHCHK();
    const bool fast = PCC::kItemsExact && fast_epilogue(k);
    // the generic pass C reads the null decisions as bits
    if (k.mask_ready && !fast) HIPCHK(hipStreamWaitEvent(st, k.mask_ready, 0));
    tk_begin(TK_COLC, st);
    if (fast) {
        if constexpr (PCC::kItemsExact) {
            if constexpr (N1 == 2048 && N2 % 16 == 0)
                k_pairC_fast32<PairCols<N1, 16, 512, CF, CI, -1>, 512>
                    <<<dim3((unsigned)(N2 / 16), (unsigned)k.npairs), dim3(512), 0, st>>>(k);
            else
                k_pairC_fast<PCC, TC><<<dim3((unsigned)(N2 / BC), (unsigned)k.npairs), dim3(TC), 0, st>>>(k);
        }
    } else if (PC::kRegCols && fold_epilogue(k)) {
        if constexpr (PC::kRegCols) {
            // 128 columns per workgroup: the lane-private LDS staging of the
            // column (N1 x 8 B per lane) then allows ~5 workgroups per CU
            constexpr int FB = B > 128 ? 128 : B;
            using PCF = PairCols<N1, FB, FB, CF, CI>;
            k_pairC_fold<PCF, FB><<<dim3((unsigned)(N2 / FB), (unsigned)k.npairs), dim3(FB), 0, st>>>(k);
        }
    } else {
        k_pairC<PC, T><<<gc, dim3(T), 0, st>>>(k);
    }
    tk_end(st);
    LAUNCHCHK();
    if (fast && k.mtab) {
        if (k.mask_ready) HIPCHK(hipStreamWaitEvent(st, k.mask_ready, 0));
        tk_begin(TK_NULLFIX, st);
        // grid-stride over the word list: ~1/8 of the words per channel
        const unsigned gx = (unsigned)((k.N / 32 / 8 + 255) / 256);
        k_null_fix_list<<<dim3(gx ? gx : 1, (unsigned)k.p.nchan), dim3(256), 0, st>>>(k);
        tk_end(st);
        LAUNCHCHK();
    }
    return PSS_OK;
}

static int run_fourstep(KP &k, hipStream_t st, const float *mask_row) {
    const int64_t N = k.N;
    if (N == (1 << 22)) {
        // C3: 1024 x 4096 (two 4096-point rows of a pair in 66 KB: two row
        // workgroups per CU; 16-column pass-C blocks, 64-B output segments)
        k.N2 = 4096;
        k.N1 = 1024;
        return launch_pair<1024, 8, 512, C1kF, C1kF, 4096, 512, C4k, C4k, 256, kBC, kTC>(k, st, mask_row);
    }
    if (N == (1 << 23)) {
        k.N2 = 8192;
        k.N1 = 1024;
        return launch_pair<1024, 8, 512, C1kF, C1kF, 8192, 1024, C8kF, C8kI, 512>(k, st, mask_row);
    }
    if (N == (1 << 24)) {
        if (k.p.null_mode != PSS_NULL_DELAYED && !k.p.htab && !k.p.tail_a) {
            // C5: 1024 x 16384 -- C3's column kernels (1024-point columns:
            // pass A two workgroups per CU, pass C 16-column blocks) and a
            // one-row-at-a-time 16384-point row pass (PairRowsSeq, 1024
            // threads, 133 KB of LDS)
            k.N2 = 16384;
            k.N1 = 1024;
            return launch_pair<1024, 8, 512, C1kF, C1kF, 16384, 1024, C16kF, C16kI, 1024, kBC, kTC>(k, st, mask_row);
        }
        // with a delayed null (the mask table's row engine holds a pair of
        // rows), a transfer function or the tail: 2048 x 8192.  Pass A: the
        // LDS-staged fast kernel on 2048-point columns; pass C: 16-column
        // register-resident blocks (passC_fast32)
        k.N2 = 8192;
        k.N1 = 2048;
        return launch_pair<2048, 8, 512, C2kF, C2kF, 8192, 1024, C8kF, C8kI, 512, 8, 1024>(k, st, mask_row);
    }
    if (N >= (1 << 17)) {
        // 2^17 .. 2^21: rows of 4096 (the C3 row kernel: two rows of a pair
        // in 66 KB, two workgroups per CU) and N / 4096 columns; the column
        // kernels keep their 8192 / N1-column blocks (N2 / B >= 16 per pair)
        k.N2 = 4096;
        k.N1 = N / 4096;
        switch (k.N1) {
#define CASE4K(N1_, CF, CI)                                                                          \
    case N1_:                                                                                        \
        return launch_pair<N1_, 8192 / N1_, 512, CF, CF, 4096, 512, C4k, C4k, 256>(k, st, mask_row);
            CASE4K(32, C32F, C32I)
            CASE4K(64, C64F, C64I)
            CASE4K(128, C128F, C128I)
            CASE4K(256, C256, C256)
            CASE4K(512, C512F, C512I)
#undef CASE4K
            default: break;
        }
        return fail(PSS_EUNSUPPORTED, "four-step: N=%lld", (long long)N);
    }
    // 2^14 .. 2^16: N1 = 16 columns, rows of N/16
    k.N1 = 16;
    k.N2 = N / 16;
    switch (k.N2) {
        case 1024:
            return launch_pair<16, 512, 512, C16, C16, 1024, 128, C1kF, C1kI, 64>(k, st, mask_row);
        case 2048:
            return launch_pair<16, 512, 512, C16, C16, 2048, 256, C2kF, C2kI, 128>(k, st, mask_row);
        case 4096:
            return launch_pair<16, 512, 512, C16, C16, 4096, 512, C4k, C4k, 256>(k, st, mask_row);
        default: break;
    }
    return fail(PSS_EUNSUPPORTED, "four-step: N=%lld", (long long)N);
}

// Mixed-radix four-step (see smooth_split): columns of N1 in registers (one
// column per thread, B = T columns per workgroup), rows by the power-of-two
// row engine.  Generic (looped) column kernels; no mask table.
template <int N1, typename CF, typename CI, int T>
static int launch_smooth_n2(KP &k, hipStream_t st) {
    switch (k.N2) {
        case 1024: return launch_pair<N1, T, T, CF, CI, 1024, 128, C1kF, C1kI, 64>(k, st, nullptr);
        case 2048: return launch_pair<N1, T, T, CF, CI, 2048, 256, C2kF, C2kI, 128>(k, st, nullptr);
        case 4096: return launch_pair<N1, T, T, CF, CI, 4096, 512, C4k, C4k, 256>(k, st, nullptr);
        case 8192: return launch_pair<N1, T, T, CF, CI, 8192, 1024, C8kF, C8kI, 512>(k, st, nullptr);
        default: return fail(PSS_EUNSUPPORTED, "mixed-radix four-step: N2=%lld", (long long)k.N2);
    }
}

static int run_smooth(KP &k, hipStream_t st) {
    int64_t n1 = 0, n2 = 0;
    if (!smooth_split(k.N, &n1, &n2)) return fail(PSS_EUNSUPPORTED, "N=%lld", (long long)k.N);
    k.N1 = n1;
    k.N2 = n2;
    if (n1 == 1250 && n2 == 2500) {
        // 4-column blocks (2500 = 4 x 625) of 250 threads, 20 values each
        using C1250 = RList<2, 5, 5, 5, 5>;
        return launch_pair<1250, 4, 250, C1250, C1250, 2500, 250, RList<5, 5, 5, 5, 4>, RList<4, 5, 5, 5, 5>, 250, 4,
                           250>(k, st, nullptr);
    }
    switch (n1) {
        case 6:  return launch_smooth_n2<6, RList<2, 3>, RList<3, 2>, 256>(k, st);
        case 10: return launch_smooth_n2<10, RList<2, 5>, RList<5, 2>, 256>(k, st);
        case 12: return launch_smooth_n2<12, RList<4, 3>, RList<3, 4>, 256>(k, st);
        case 20: return launch_smooth_n2<20, RList<4, 5>, RList<5, 4>, 256>(k, st);
        case 24: return launch_smooth_n2<24, RList<2, 4, 3>, RList<3, 4, 2>, 256>(k, st);
        case 30: return launch_smooth_n2<30, RList<2, 3, 5>, RList<5, 3, 2>, 256>(k, st);
        case 40: return launch_smooth_n2<40, RList<2, 4, 5>, RList<5, 4, 2>, 128>(k, st);
        case 48: return launch_smooth_n2<48, RList<4, 4, 3>, RList<3, 4, 4>, 128>(k, st);
        case 60: return launch_smooth_n2<60, RList<4, 3, 5>, RList<5, 3, 4>, 128>(k, st);
        default: return fail(PSS_EUNSUPPORTED, "N1=%lld", (long long)n1);
    }
}

static int run_single(KP &k, hipStream_t st) {
    k.N1 = 1;
    k.N2 = k.N;
    switch (k.N) {
        case 64: return launch_single<64, 64, 256, C64F, C64I>(k, st);
        case 128: return launch_single<128, 32, 256, C128F, C128I>(k, st);
        case 256: return launch_single<256, 16, 256, C256, C256>(k, st);
        case 512: return launch_single<512, 8, 256, C512F, C512I>(k, st);
        case 1024: return launch_single<1024, 4, 256, C1kF, C1kI>(k, st);
        case 2048: return launch_single<2048, 2, 256, C2kF, C2kI>(k, st);
        case 4096: return launch_single<4096, 1, 256, C4k, C4k>(k, st);
        case 8192: return launch_single<8192, 1, 512, C8kF, C8kI>(k, st);
        default: break;
    }
    return fail(PSS_EUNSUPPORTED, "single-pass: N=%lld", (long long)k.N);
}

template <int L, typename R>
static int bs_col(const KP &k, const BsArgs &a, int rows, int kind, hipStream_t st) {
    dim3 g((unsigned)(a.M2 / (8192 / L)), (unsigned)rows);
    if (kind == 0) k_bs_col<L, R, 0><<<g, dim3(256), 0, st>>>(k, a);
    else if (kind == 1) k_bs_col<L, R, 1><<<g, dim3(256), 0, st>>>(k, a);
    else if (kind == 2) k_bs_col<L, R, 2><<<g, dim3(256), 0, st>>>(k, a);
    else if constexpr (L <= 2048) {
        if (kind == 3) k_bs_col<L, R, 3><<<g, dim3(256), 0, st>>>(k, a);
        else k_bs_col<L, R, 4><<<g, dim3(256), 0, st>>>(k, a);
    } else {
        return fail(PSS_EUNSUPPORTED, "Bluestein: fused pair passes need M1 <= 2048");
    }
    LAUNCHCHK();
    return PSS_OK;
}

static int bs_col_any(const KP &k, const BsArgs &a, int rows, int inv, hipStream_t st) {
    switch (a.M1) {
        case 8:    return bs_col<8, RList<8>>(k, a, rows, inv, st);
        case 16:   return bs_col<16, RList<16>>(k, a, rows, inv, st);
        case 32:   return bs_col<32, RList<2, 16>>(k, a, rows, inv, st);
        case 64:   return bs_col<64, RList<4, 16>>(k, a, rows, inv, st);
        case 128:  return bs_col<128, RList<8, 16>>(k, a, rows, inv, st);
        case 256:  return bs_col<256, RList<16, 16>>(k, a, rows, inv, st);
        case 512:  return bs_col<512, RList<2, 16, 16>>(k, a, rows, inv, st);
        case 1024: return bs_col<1024, RList<4, 16, 16>>(k, a, rows, inv, st);
        case 2048: return bs_col<2048, RList<8, 16, 16>>(k, a, rows, inv, st);
        case 4096: return bs_col<4096, RList<16, 16, 16>>(k, a, rows, inv, st);
        default: return fail(PSS_EUNSUPPORTED, "Bluestein: M1=%lld", (long long)a.M1);
    }
}

static int bs_row_any(const KP &k, const BsArgs &a, int rows, hipStream_t st) {
    dim3 g((unsigned)a.M1, (unsigned)rows);
    if (a.M2 == 4096) {
        using RW = BsRow<4096, RList<16, 16, 16>, RList<16, 16, 16>>;
        k_bs_row<RW><<<g, dim3(RW::T), 0, st>>>(k, a);
    } else if (a.M2 == 8192) {
        using RW = BsRow<8192, RList<16, 16, 16, 2>, RList<2, 16, 16, 16>>;
        k_bs_row<RW><<<g, dim3(RW::T), 0, st>>>(k, a);
    } else {
        return fail(PSS_EUNSUPPORTED, "Bluestein: M2=%lld", (long long)a.M2);
    }
    LAUNCHCHK();
    return PSS_OK;
}

// forward DFT -> delay ramp / transfer function -> inverse DFT / N of every
// channel row, in place in src, channel batches of nb through the Z buffer:
// 5 passes over M (first col, row, fused middle col, row, last col)
static int bs_filter(const KP &k, BsArgs a, int64_t nb, hipStream_t st) {
    for (int64_t r0 = 0; r0 < k.p.nchan; r0 += nb) {
        const int rows = (int)((k.p.nchan - r0) < nb ? (k.p.nchan - r0) : nb);
        a.r0 = (int)r0;
        int rc = bs_col_any(k, a, rows, 0, st);
        if (!rc) rc = bs_row_any(k, a, rows, st);
        if (!rc) rc = bs_col_any(k, a, rows, 2, st);
        if (!rc) rc = bs_row_any(k, a, rows, st);
        if (!rc) rc = bs_col_any(k, a, rows, 1, st);
        if (rc) return rc;
    }
    return PSS_OK;
}

// Pair runs: forward DFT (X in src, natural order) -> channel separation,
// ramps, recombination (k_bs_sep) -> inverse DFT / N, per batch of nb pair
// rows: 6 passes over M and one over N instead of 5 over M for each of the
// two channels.
static bool bs_fused(const BsArgs &a) { return a.M1 <= 2048; }   // 8192 / M1 >= 4 columns per block

static int bs_filter_pair(const KP &k, BsArgs a, int64_t nb, int npairs, hipStream_t st) {
    const bool fused = bs_fused(a);
    for (int64_t r0 = 0; r0 < npairs; r0 += nb) {
        const int rows = (int)((npairs - r0) < nb ? (npairs - r0) : nb);
        a.r0 = (int)r0;
        BsArgs f = a, g = a;
        f.mode = 4;                 // forward: ..., X -> src (consumed by its first pass)
        f.dst = const_cast<cf *>(a.src);
        g.mode = 3;                 // inverse: conj(Y) w -> ..., result -> dst
        // (fused: the first pass generates the source, the last runs the epilogue)
        int rc = bs_col_any(k, a, rows, fused ? 3 : 0, st);
        if (!rc) rc = bs_row_any(k, a, rows, st);
        if (!rc) rc = bs_col_any(k, f, rows, 1, st);
        // (the separation as its own kernel: fused into the inverse's first
        // pass, which reads X_n and X_{N-n}, each sample computed both
        // channels' ramps at its bin -- twice sep's ramp work at two
        // workgroups per CU: 2.74 ms against 0.79 + 0.90 at 512 x (2^20 - 2))
        if (!rc) {
            k_bs_sep<<<dim3((unsigned)std::min<int64_t>((k.N / 2 + 256) / 256, 1024), (unsigned)rows), dim3(256), 0,
                       st>>>(k, const_cast<cf *>(a.src), a.ld, (int)r0);
            HIPCHK(hipGetLastError());
        }
        if (!rc) rc = bs_col_any(k, g, rows, 0, st);
        if (!rc) rc = bs_row_any(k, g, rows, st);
        g.mode = 1;
        if (!rc) rc = bs_col_any(k, g, rows, fused ? 4 : 1, st);
        if (rc) return rc;
    }
    return PSS_OK;
}

// The float64 null decisions of the packed paths (k_null_refine), between
// the inverse transform (W1 = data + i mask per row) and the epilogue.
static bool refine_null(const KP &k) {
    return k.p.null_mode == PSS_NULL_DELAYED && (k.N & 1) == 0 && k.N <= kRefineMaxN && !k.p.tail_a &&
           !k.p.htab && !(g_flags & PSS_FLAG_NULL_F32);
}

static int launch_null_refine(KP &k, hipStream_t st) {
    const WsLayout w = ws_layout(k.p.nchan, k.N, k.p.htab != nullptr);
    char *base = reinterpret_cast<char *>(k.p.work);
    cf *W1 = reinterpret_cast<cf *>(base);
    double2 *tw = reinterpret_cast<double2 *>(base + w.rf_tw);
    double2 *B = reinterpret_cast<double2 *>(base + w.rf_B);
    unsigned int *mx = reinterpret_cast<unsigned int *>(base + w.rf_mx);
    const float *box = k.p.inj_box;
    if (!box) {
        float *row = reinterpret_cast<float *>(base + w.row);
        k_box_row<<<stream_grid(k.N, 1), dim3(256), 0, st>>>(k, row);
        LAUNCHCHK();
        box = row;
    }
    k_tw64<<<stream_grid(k.N, 1), dim3(256), 0, st>>>(k.N, tw);
    LAUNCHCHK();
    double2 *part = reinterpret_cast<double2 *>(base + w.rf_part);
    unsigned long long *list = reinterpret_cast<unsigned long long *>(base + w.rf_list);
    unsigned int *cnt = reinterpret_cast<unsigned int *>(base + w.rf_cnt);
    const int64_t K = k.N / 2 + 1, cap = (g_flags & PSS_FLAG_REFINE_PER_SAMPLE) ? 0 : refine_cap(k.p.nchan, k.N);
    k_null_bspec<<<dim3((unsigned)((K + 255) / 256), (unsigned)kBsParts), dim3(256), 0, st>>>(box, k.N, tw, part);
    LAUNCHCHK();
    k_null_bsum<<<dim3((unsigned)((K + 255) / 256)), dim3(256), 0, st>>>(part, K, B);
    LAUNCHCHK();
    HIPCHK(hipMemsetAsync(mx, 0, (size_t)k.p.nchan * 4, st));
    HIPCHK(hipMemsetAsync(cnt, 0, 4, st));
    k_row_absmax<<<dim3((unsigned)std::min<int64_t>(64, (k.N + 255) / 256), (unsigned)k.p.nchan), dim3(256), 0, st>>>(
        W1, k.N, mx);
    LAUNCHCHK();
    const dim3 gs((unsigned)((k.N + 255) / 256), (unsigned)k.p.nchan);
    k_null_cands<<<gs, dim3(256), 0, st>>>(k, W1, mx, list, cnt, cap);
    LAUNCHCHK();
    k_null_refine_list<<<dim3(4096), dim3(256), 0, st>>>(k, W1, B, list, cnt, cap);
    LAUNCHCHK();
    k_null_refine<<<gs, dim3(256), 0, st>>>(k, W1, B, mx, cnt, cap);     // (overflow only)
    LAUNCHCHK();
    return PSS_OK;
}

static int run_bluestein(KP &k, hipStream_t st) {
    const WsLayout w = ws_layout(k.p.nchan, k.N, k.p.htab != nullptr);
    const BsGeom g = bs_geom(k.p.nchan, k.N);
    char *base = reinterpret_cast<char *>(k.p.work);
    cf *W1 = reinterpret_cast<cf *>(base);
    BsArgs a;
    memset(&a, 0, sizeof(a));
    a.chirp = reinterpret_cast<const cf *>(base + w.bs_chirp);
    a.bhat = reinterpret_cast<const cf *>(base + w.bs_bhat);
    a.N = k.N;
    a.ld = k.N;
    a.fastio = !(g_flags & PSS_FLAG_NO_FAST);
    a.M = g.M;
    a.M1 = g.M1;
    a.M2 = g.M2;
    // two channels per complex row unless a delayed null rides in the
    // imaginary part (its mask shares the channel's transform)
    const bool pair = k.p.null_mode != PSS_NULL_DELAYED;
    k.poff = k.p.chan0 & 1;                 // pairs of (even, odd) GLOBAL channels: shard invariant
    k.npairs = (k.p.nchan + k.poff + 1) / 2;
    dim3 ge = stream_grid((k.N + 3) / 4, pair ? k.npairs : k.p.nchan);
    const bool fused = pair && g.M1 <= 2048;      // (bs_fused)
    // fused pair runs: W1's rows are internal (no source / epilogue kernel
    // reads them), so they may start on 128-B lines where W1 has the room
    const int64_t ldp = (k.N + 15) & ~(int64_t)15;
    if (fused && k.npairs * ldp <= (int64_t)k.p.nchan * k.N) a.ld = ldp;
    tk_begin(TK_FALLBACK, st);
    if (!pair) k_fb_source<<<ge, dim3(256), 0, st>>>(k);
    else if (!fused) k_fb_source_pair<<<ge, dim3(256), 0, st>>>(k);
    LAUNCHCHK();
    k_bs_chirp<<<stream_grid(k.N, 1), dim3(256), 0, st>>>(reinterpret_cast<cf *>(base + w.bs_chirp), k.N);
    LAUNCHCHK();
    BsArgs b = a;                       // Bhat: generate b, forward transform, 1/M
    b.mode = 2;
    b.Z = reinterpret_cast<cf *>(base + w.bs_bhat);
    int rc = bs_col_any(k, b, 1, 0, st);
    if (!rc) rc = bs_row_any(k, b, 1, st);
    if (rc) return rc;
    a.Z = reinterpret_cast<cf *>(base + w.bs_z);
    a.src = W1;
    a.dst = W1;
    a.mode = 0;
    if (pair) {
        if ((rc = bs_filter_pair(k, a, g.nb, k.npairs, st))) return rc;
        if (!fused) k_fb_epilogue_pair<<<ge, dim3(256), 0, st>>>(k);
        tk_end(st);
        LAUNCHCHK();
        return PSS_OK;
    }
    if ((rc = bs_filter(k, a, g.nb, st))) return rc;
    if (refine_null(k) && (rc = launch_null_refine(k, st))) return rc;
    k_fb_epilogue<<<ge, dim3(256), 0, st>>>(k);
    tk_end(st);
    LAUNCHCHK();
    return PSS_OK;
}

static int run_fallback(KP &k, hipStream_t st) {
    if (bs_len(k.N) && !(g_flags & PSS_FLAG_DIRECT_DFT)) return run_bluestein(k, st);
    dim3 g = stream_grid((k.N + 3) / 4, k.p.nchan);
    tk_begin(TK_FALLBACK, st);
    k_fb_source<<<g, dim3(256), 0, st>>>(k);
    LAUNCHCHK();
    k_fb_twiddles<<<stream_grid(k.N, 1), dim3(256), 0, st>>>(k);
    LAUNCHCHK();
    dim3 gd((unsigned)((k.N + 255) / 256), (unsigned)k.p.nchan);
    k_fb_dft<false><<<gd, dim3(256), 0, st>>>(k);
    LAUNCHCHK();
    k_fb_dft<true><<<gd, dim3(256), 0, st>>>(k);
    LAUNCHCHK();
    if (refine_null(k)) {
        const int rc = launch_null_refine(k, st);
        if (rc) return rc;
    }
    k_fb_epilogue<<<g, dim3(256), 0, st>>>(k);
    tk_end(st);
    LAUNCHCHK();
    return PSS_OK;
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
        dim3 g = stream_grid((k.N + 3) / 4, p->nchan);
        tk_begin(TK_ELEM, st);
        k_elementwise<<<g, dim3(256), 0, st>>>(k);
        tk_end(st);
        LAUNCHCHK();
        return PSS_OK;
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

// odd n: forward N-point direct DFT x ramp, then the (N - 1)-point inverse
static int shift_rows_odd(float *rows, int32_t nrows, int64_t n, int64_t ld, const uint64_t *ramp, void *work,
                          hipStream_t st) {
    if (n < 3) return fail(PSS_EINVAL, "shift_t: invalid number of data points (%lld) for the inverse", (long long)(n - 1));
    if (!ramp || !work || !rows) return fail(PSS_EINVAL, "shift_t: NULL argument");
    if (nrows > 65535) return fail(PSS_EINVAL, "nchan %d > 65535 per launch", nrows);
    KP k;
    memset(&k, 0, sizeof(k));
    k.p.nchan = nrows;
    k.p.nsamp = n;
    k.p.ld = ld;
    k.p.data = rows;
    k.p.work = work;
    k.p.src = PSS_SRC_LOAD;
    k.p.shift = 1;
    k.p.data_in_fft = 1;
    k.p.ramp = ramp;
    k.N = n;
    k.N1 = 1;
    k.N2 = n;
    const WsLayout w = ws_layout(nrows, n);
    cf *tw = reinterpret_cast<cf *>(reinterpret_cast<char *>(work) + w.odd_tw);
    dim3 g = stream_grid((n + 3) / 4, nrows);
    k_fb_source<<<g, dim3(256), 0, st>>>(k);
    LAUNCHCHK();
    k_fb_twiddles<<<stream_grid(n, 1), dim3(256), 0, st>>>(k);
    LAUNCHCHK();
    k_odd_twiddles<<<stream_grid(n - 1, 1), dim3(256), 0, st>>>(tw, n - 1);
    LAUNCHCHK();
    // only bins 0..M of the forward transform are used
    const int64_t M = (n - 1) / 2;
    k_fb_dft<false><<<dim3((unsigned)((M + 1 + 255) / 256), (unsigned)nrows), dim3(256), 0, st>>>(k);
    LAUNCHCHK();
    k_odd_irfft<<<dim3((unsigned)((n - 1 + 255) / 256), (unsigned)nrows), dim3(256), 0, st>>>(k, tw, rows, ld);
    LAUNCHCHK();
    return PSS_OK;
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
