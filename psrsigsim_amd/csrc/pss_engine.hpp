#pragma once
// pss_engine.hpp -- device code and launch templates of the MI355X engine (gfx950),
// shared by the launch units (pss_pipeline.hip, pss_fourstep.hip, pss_smooth.hip,
// pss_single.hip, pss_fallback.hip).
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
#include <algorithm>

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
// error reporting and opt-in per-kernel timing (defined in pss_pipeline.hip)
// ---------------------------------------------------------------------------
int fail(int code, const char *fmt, ...);

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

enum { TK_ELEM = 0, TK_SINGLE, TK_COLA, TK_ROW, TK_COLC, TK_FALLBACK, TK_NULLFIX, TK_N };
void tk_begin(int kind, hipStream_t st);
void tk_end(hipStream_t st);
// launch-plan log (pss_plan_collect): every launch path notes the kernels it
// picked ("fourstep 1024x4096 A:fast R:pair_row C:fast N:fix_list"), so the
// parity tests can assert which kernels produced the bits they check
void plan_note(const char *fmt, ...);

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
    // single-workgroup kernel with a float64-refined delayed null: the
    // inverse transform's (data, mask) pairs go to this [nchan][N] buffer
    // (the packed paths' W1) instead of through the epilogue
    cf *w1_out;
    // shared-profile fast pass A: the pulse profile at every sample, in the
    // pass's item order (k_prof_cols, PairCols::prof_cols)
    const float4 *pcol;
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
// shared-profile fast pass A reads the per-run sample table (PairCols::prof_cols)
#ifndef PSS_PCOL
#define PSS_PCOL 1
#endif
static constexpr bool kPcol = PSS_PCOL != 0;

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
// The atomics land in the hardware's order: the pieces are fp32 sums of one
// row's samples, so their float64 sum is exact (order-free) unless a window
// mixes pieces ~2^29 apart in magnitude, and a last-bit difference of the
// float64 mean changes the float32 / int8 result only at a rounding boundary
// (tests/test_gpu_observe_resample.py: two identical runs, the same bits).
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
            if (k.w1_out) {
                // (data, mask) for the float64 null refine; the epilogue runs
                // after it (k_fb_epilogue, as on the other packed paths)
                cf *w = k.w1_out + (int64_t)(r0 + b) * L + n0;
#pragma unroll
                for (int i = 0; i < 4; ++i) w[i] = make_float2(pre[i], msk[i]);
            } else {
                epilogue4(k, r0 + b, n0, 4, pre, msk, !re_in);
            }
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

    // Pass A's 4-sample item it of a column block: row n1, first column b4.
    // Lanes = consecutive rows n1 (of one 4-column group where N1 % 64 == 0):
    // the transposed LDS writes are conflict-free.
    __device__ static __forceinline__ void item_of(int it, int &n1, int &b4) {
        if constexpr (N1 % 64 == 0) {
            n1 = it % N1;
            b4 = (it / N1) * 4;
        } else {
            n1 = it / (B / 4);
            b4 = (it - n1 * (B / 4)) * 4;
        }
    }

    // The shared profile (prof_rows == 1: one PCHIP row for every channel,
    // e.g. C3's GaussProfile) is a function of the sample alone, so it is
    // evaluated once per run instead of once per pair: entry cbx (N1 B / 4) +
    // it holds samples n .. n + 3 of item it of column block cbx, so each
    // pass-A workgroup reads one contiguous 4 N1 B-byte block (a wave 1 KB per
    // item) in place of a phase walk, an LDS gather and a cubic per sample.
    // The same integer walk and the same fused cubic as the per-pair form:
    // bitwise its values.
    __device__ static void prof_cols(const KP &k, float4 *out) {
        const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (e >= k.N / 4) return;
        constexpr int IPB = N1 * B / 4;                 // items per column block
        const int cbx = (int)(e / IPB), it = (int)(e - (int64_t)cbx * IPB);
        int n1, b4;
        item_of(it, n1, b4);
        const PssPipeline &p = k.p;
        const uint32_t n = (uint32_t)(n1 * (int)k.N2) + (uint32_t)(cbx * B) + (uint32_t)b4;   // N < 2^24
        uint32_t dlo;
        uint64_t dhi;
        phase_delta(p, dlo, dhi);
        const float4 *prof = reinterpret_cast<const float4 *>(p.prof);
        PhaseWalk w;
        w.start(p, n);
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t iv;
            float u;
            if (i) w.step(dlo, dhi, p.knot_m);
            w.get_full(iv, u);
            const float4 A = prof[iv];
            v[i] = fmaf(fmaf(fmaf(A.x, u, A.y), u, A.z), u, A.w);
        }
        out[e] = make_float4(v[0], v[1], v[2], v[3]);
    }

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
        if constexpr (FAST && SHARED && kPcol) {
            // the profile from the per-run sample table (prof_cols): loads
            // issued first, under the Philox draws
            const float dna = hasa ? p.draw_norm : 0.f, dnb = hasb ? p.draw_norm : 0.f;
            const float4 *pc = k.pcol + (int64_t)cbx * (N1 * B / 4);
            float4 P[ITEMS];
#pragma unroll
            for (int t = 0; t < ITEMS; ++t) P[t] = pc[tid + t * T];
#pragma unroll
            for (int t = 0; t < ITEMS; ++t) {
                const int it = tid + t * T;
                int n1, b4;
                item_of(it, n1, b4);
                const uint32_t n = (uint32_t)(n1 * (int)N2) + (uint32_t)n20 + (uint32_t)b4;   // N < 2^24
                const float4 qa = chi2_1x4(g.bits(n >> 2, ca, 0u), dna);
                const float4 qb = chi2_1x4(g.bits(n >> 2, cb, 0u), dnb);
                const float pv[4] = {P[t].x, P[t].y, P[t].z, P[t].w};
                const float va[4] = {qa.x, qa.y, qa.z, qa.w}, vb[4] = {qb.x, qb.y, qb.z, qb.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) lds[LdsC::at(b4 + i, n1)] = make_float2(pv[i] * va[i], pv[i] * vb[i]);
            }
        } else if constexpr (FAST) {
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
template <typename C>
__global__ __launch_bounds__(256) void k_prof_cols(KP k, float4 *out) { C::prof_cols(k, out); }
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


// ---------------------------------------------------------------------------
// entry points of the launch units (one translation unit each, compiled in
// parallel: psrsigsim_amd/build.py)
// ---------------------------------------------------------------------------
int launch_elementwise(const KP &k, hipStream_t st);              // pss_pipeline.hip
int launch_null_fix(const KP &k, hipStream_t st);                 // pss_fourstep.hip
int run_fourstep(KP &k, hipStream_t st, const float *mask_row);   // pss_fourstep.hip
int run_smooth(KP &k, hipStream_t st);                            // pss_smooth.hip (N1 = 6 .. 20)
int run_smooth_b(KP &k, hipStream_t st);                          // pss_smooth_b.hip (N1 = 24, 30, 40)
int run_smooth_c(KP &k, hipStream_t st);                          // pss_smooth_c.hip (N1 = 48, 60; 1250 x 2500)
int run_fourstep_b(KP &k, hipStream_t st, const float *mask_row); // pss_fourstep_b.hip (N != 2^22)
int run_single(KP &k, hipStream_t st);                            // pss_single.hip
int run_fallback(KP &k, hipStream_t st);                          // pss_fallback.hip
int launch_null_refine(KP &k, hipStream_t st);                    // pss_fallback.hip
int launch_fb_epilogue(KP &k, hipStream_t st);                    // pss_fallback.hip
int shift_rows_odd(float *rows, int32_t nrows, int64_t n, int64_t ld, const uint64_t *ramp, void *work,
                   hipStream_t st);                               // pss_fallback.hip
// the mask-table template's (build_mask_table) non-template kernels, launched
// through pss_fourstep.hip (each kernel is compiled in one unit only)
int launch_node_params(uint64_t *ramp, float *nyq, int L, hipStream_t st);
int launch_mask_table(const float *nodes, int64_t N, uint2 *bits, uint32_t *base, float *coef, uint32_t *counter,
                      hipStream_t st);
int launch_mask_words(const uint2 *bits, uint32_t nwords, uint32_t *list, uint32_t *count, hipStream_t st);
int launch_mask_bits(const KP &k, uint32_t *bm, hipStream_t st);

// ---------------------------------------------------------------------------
// host dispatch
// ---------------------------------------------------------------------------
static inline bool is_pow2(int64_t n) { return n > 0 && (n & (n - 1)) == 0; }

static inline dim3 stream_grid(int64_t items, int rows) {
    int64_t bx = (items + 255) / 256;
    if (bx > 4096) bx = 4096;
    if (bx < 1) bx = 1;
    return dim3((unsigned)bx, (unsigned)rows, 1);
}


template <int L, int BATCH, int T, typename F, typename I>
static int launch_single(const KP &k, hipStream_t st) {
    using SP = SinglePass<L, BATCH, T, F, I>;
    dim3 grid((k.p.nchan + BATCH - 1) / BATCH);
    plan_note("single %d", L);
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

extern int g_flags;   // pss_set_flags (test hook), pss_pipeline.hip

// Bluestein geometry of a fallback length N > 8192 (path 3b): M = M1 x M2,
// nb channels per convolution batch (the batch buffer is about one W buffer).
struct BsGeom { int64_t M, M1, M2, nb; };
static inline bool bs_len(int64_t N) { return N > 8192 && N <= (1ll << 24); }
static inline BsGeom bs_geom(int32_t nchan, int64_t N) {
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
    int64_t pcol;                      // four-step: the profile at every sample (float4 items, k_prof_cols)
};

static inline WsLayout ws_layout(int32_t nchan, int64_t N, bool filt = false) {
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
        w.pcol = o;  o += al256(N * 4);                        // shared-profile pass A: profile per sample
    } else if (!filt && is_pow2(N) && N >= 64 && N <= 8192) {
        // single-workgroup lengths: W1 [nchan][N] cf and the float64 null
        // refine's buffers (a delayed null: run_single)
        o += al256((int64_t)nchan * N * 8);
        w.rf_tw = o; o += al256(N * 16);
        w.rf_B = o;  o += al256((N / 2 + 1) * 16);
        w.rf_mx = o; o += al256((int64_t)nchan * 4);
        w.rf_part = o; o += al256((int64_t)kBsParts * (N / 2 + 1) * 16);
        w.rf_list = o; o += al256(refine_cap(nchan, N) * 8);
        w.rf_cnt = o;  o += 256;
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
            w.pcol = o; o += al256(N * 4);
        }
    }
    w.row = o;
    o += al256(N * 4);
    w.total = o;
    return w;
}

// The float64 null decisions of the packed paths (k_null_refine): the
// direct / Bluestein rows and the single-workgroup kernel's, between the
// inverse transform (W1 = data + i mask per row) and the epilogue.
static inline bool refine_null(const KP &k) {
    return k.p.null_mode == PSS_NULL_DELAYED && (k.N & 1) == 0 && k.N <= kRefineMaxN && !k.p.tail_a &&
           !k.p.htab && !(g_flags & PSS_FLAG_NULL_F32);
}

// Fast-path selection (kernels specialised for the north-star configuration;
// results are bitwise identical to the generic kernels).

static inline bool fast_source(const PssPipeline &p) {
    if (g_flags & PSS_FLAG_NO_FAST) return false;
    // (nint == knot_m: the table spans the period, so the fast walk needs no
    // extrapolation clamp -- pulsar._device_table always builds it so)
    return p.src == PSS_SRC_SEARCH && !p.gen_amp && p.gen_df == 1.0f && !p.inj_gen && p.null_mode != PSS_NULL_UNDELAYED &&
           p.nint <= kFastNint && !p.prof_split && (uint32_t)p.nint == p.knot_m;
}
// Fold-mode fast passes of the mixed-radix split (PairCols::passA_fold /
// passC_fold): the fold source with chi2(df != 1) pair draws, and an
// epilogue of noise only (any df != 1), no injected draws.
static inline bool fold_source(const PssPipeline &p) {
    if (g_flags & PSS_FLAG_NO_FAST) return false;
    return p.src == PSS_SRC_FOLD && !p.gen_amp && !p.inj_gen && p.gen_df != 1.0f && p.nph > 0 &&
           p.null_mode != PSS_NULL_UNDELAYED;
}
static inline bool fold_epilogue(const KP &k) {
    const PssPipeline &p = k.p;
    if (g_flags & PSS_FLAG_NO_FAST) return false;
    if (p.out_kind != PSS_OUT_NONE || p.inj_noise || p.inj_rep) return false;
    return p.noise && p.noise_df != 1.0f && p.null_mode != PSS_NULL_DELAYED;
}
static inline bool fast_epilogue(const KP &k) {
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
static inline int build_mask_table(KP &k, hipStream_t st, const float *mask_row, char *w, const WsLayout &L) {
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
    if (const int rc = launch_node_params(nramp, nnyq, log2n, st)) return rc;
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
    if (const int rc = launch_mask_table(nodes, k.N, reinterpret_cast<uint2 *>(w + L.bits),
                                         reinterpret_cast<uint32_t *>(w + L.base), reinterpret_cast<float *>(w + L.coef),
                                         counter, st))
        return rc;
    {
        uint32_t *wl = reinterpret_cast<uint32_t *>(w + L.wlist);
        uint32_t *wcount = reinterpret_cast<uint32_t *>(w + L.misc + 8);
        HIPCHK(hipMemsetAsync(wcount, 0, 4, st));
        const uint32_t nwords = (uint32_t)(k.N / 32);
        if (const int rc = launch_mask_words(k.mt_bits, nwords, wl, wcount, st)) return rc;
        k.wlist = wl;
        k.nwlist = wcount;
    }
    k.mtab = 1;
    plan_note(" N:table");
    k.log2n = log2n;
    if (k.p.data_in_fft && !fast_epilogue(k)) {   // generic pass C reads the decisions as bits
        k.mbB = B;
        uint32_t *bm = reinterpret_cast<uint32_t *>(w + L.mbits);
        if (const int rc = launch_mask_bits(k, bm, st)) return rc;
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
SideStreams *side_streams();

template <int N1, int B, int T, typename CF, typename CI, int N2, int TR, typename RF, typename RI,
          int TRF, int BC, int TC>
static int launch_pair_passes(KP &k, hipStream_t st, const float *mask_after_a = nullptr);
// Channel count up to which the side-stream mask table forks after pass A
// (beside the row pass) instead of before it (beside pass A): it costs the
// pass it runs beside ~0.4 ms either way, which at 2048 channels is even
// (46.84-46.89 vs 46.86-47.06 ms per C3 step), at 1024 channels slightly
// better after pass A (kernels 23.05-23.12 vs 23.17-23.20 ms) and at 256
// channels -- a short pass A it slowed by a quarter -- 0.12 ms per step less
// after pass A (6.52-6.56 vs 6.64-6.68 ms, profiles/r06/ab_mask/)
#ifndef PSS_MASK_AFTER_A_NCHAN
#define PSS_MASK_AFTER_A_NCHAN 1024
#endif
static constexpr int kMaskAfterANchan = PSS_MASK_AFTER_A_NCHAN;

// BC/TC: column-block width and threads of the FAST pass C (the spill layout
// does not depend on the block width, so pass C may use wider blocks than pass
// A: its output rows are written in BC-sample (4 BC-byte) segments).
template <int N1, int B, int T, typename CF, typename CI, int N2, int TR, typename RF, typename RI,
          int TRF, int BC = B, int TC = T>
static int launch_pair(KP &k, hipStream_t st, const float *mask_row) {
    using PC = PairCols<N1, B, T, CF, CI, xrs_read(B)>;
    using PCC = PairCols<N1, BC, TC, CF, CI, xrs_write(BC)>;
    using PR = PairRows<N2, TR, RF, RI>;
    plan_note(" %dx%d", N1, N2);
    k.poff = k.p.chan0 & 1;
    k.npairs = (k.p.nchan + k.poff + 1) / 2;
    char *w = reinterpret_cast<char *>(k.p.work);
    const WsLayout L = ws_layout(k.p.nchan, k.N);
    k.Yd = reinterpret_cast<cf *>(w + L.yd);
    const float *defer_mask = nullptr;
    if (k.p.null_mode == PSS_NULL_DELAYED) {
        // the mask table's position arithmetic is for N = 2^m (validate()
        // sends delayed nulls of other lengths to the direct path)
        if constexpr ((N1 & (N1 - 1)) == 0 && N2 <= 8192) {
            // With the data in the FFT and the fast passes, nothing reads the
            // table before the null fix-up: build it on a side stream next to
            // pass A (its dozen small launches then cost no time on the main
            // stream); the fix-up waits for it.
            SideStreams *ss = k.p.data_in_fft ? side_streams() : nullptr;
            if (ss && k.p.nchan <= kMaskAfterANchan) {
                defer_mask = mask_row;            // built by launch_pair_passes after pass A
                goto mask_done;
            }
            hipStream_t ms = st;
            if (ss) {
                HIPCHK(hipEventRecord(ss->ev[30], st));
                HIPCHK(hipStreamWaitEvent(ss->s[0], ss->ev[30], 0));
                ms = ss->s[0];
            }
            {
                const int rc = build_mask_table<N1, B, T, CF, CI, N2, TR, RF, RI, TRF>(k, ms, mask_row, w, L);
                if (rc) return rc;
            }
            if (ss) {
                HIPCHK(hipEventRecord(ss->ev[31], ms));
                k.mask_ready = ss->ev[31];
            }
        } else {
            return fail(PSS_EUNSUPPORTED, "delayed null on the mixed-radix or 16384-row four-step (N=%lld)",
                        (long long)k.N);
        }
    }
mask_done:
    if (!k.p.data_in_fft) {
        // only the null mask was delayed: one elementwise pass with table lookups
        return launch_elementwise(k, st);
    }
    if (!k.p.htab) {   // (a transfer-function run has no ramps)
        cf *rt = reinterpret_cast<cf *>(w + L.rtab);
        k_pair_tab<PR::RFL><<<dim3((unsigned)k.npairs), dim3(64), 0, st>>>(k.p.ramp, k.N, k.p.nchan, k.poff,
                                                                          k.npairs, rt);
        LAUNCHCHK();
        k.rtab = rt;
    }
    return launch_pair_passes<N1, B, T, CF, CI, N2, TR, RF, RI, TRF, BC, TC>(k, st, defer_mask);
}

// The passes of one pair range (after the mask table and the ramp table).
template <int N1, int B, int T, typename CF, typename CI, int N2, int TR, typename RF, typename RI,
          int TRF, int BC, int TC>
static int launch_pair_passes(KP &k, hipStream_t st, const float *mask_after_a) {
    using PC = PairCols<N1, B, T, CF, CI, xrs_read(B)>;
    using PCC = PairCols<N1, BC, TC, CF, CI, xrs_write(BC)>;
    using PR = PairRows<N2, TR, RF, RI>;
    dim3 gc((unsigned)(N2 / B), (unsigned)k.npairs);
    tk_begin(TK_COLA, st);
    bool launched = false;
    if constexpr (PC::kRegCols) {
        if (fold_source(k.p)) {
            k_pairA_fold<PC, T><<<gc, dim3(T), 0, st>>>(k);
            plan_note(" A:fold");
            launched = true;
        }
    }
    if (launched) {
    } else if constexpr (PC::kItemsExact) {
        if (fast_source(k.p)) {
            if (k.p.prof_rows == 1) {
                if constexpr (kPcol) {
                    float4 *pcol = reinterpret_cast<float4 *>(reinterpret_cast<char *>(k.p.work) +
                                                              ws_layout(k.p.nchan, k.N).pcol);
                    const int64_t ne = k.N / 4;
                    k_prof_cols<PC><<<dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st>>>(k, pcol);
                    LAUNCHCHK();
                    k.pcol = pcol;
                }
                k_pairA_fast<PC, T, true><<<gc, dim3(T), 0, st>>>(k);
            } else {
                k_pairA_fast<PC, T, false><<<gc, dim3(T), 0, st>>>(k);
            }
            plan_note(k.p.prof_rows == 1 ? " A:fast_shared" : " A:fast");
        } else {
            k_pairA<PC, T><<<gc, dim3(T), 0, st>>>(k);
            plan_note(" A:generic");
        }
    } else {
        k_pairA<PC, T><<<gc, dim3(T), 0, st>>>(k);
        plan_note(" A:generic");
    }
    tk_end(st);
    LAUNCHCHK();
    if constexpr ((N1 & (N1 - 1)) == 0 && N2 <= 8192) {
        if (mask_after_a) {
            // (kMaskAfterANchan) the mask table on the side stream from here
            SideStreams *ss = side_streams();
            char *w = reinterpret_cast<char *>(k.p.work);
            const WsLayout L = ws_layout(k.p.nchan, k.N);
            HIPCHK(hipEventRecord(ss->ev[30], st));
            HIPCHK(hipStreamWaitEvent(ss->s[0], ss->ev[30], 0));
            const int rc = build_mask_table<N1, B, T, CF, CI, N2, TR, RF, RI, TRF>(k, ss->s[0], mask_after_a, w, L);
            if (rc) return rc;
            HIPCHK(hipEventRecord(ss->ev[31], ss->s[0]));
            k.mask_ready = ss->ev[31];
        }
    }
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
        plan_note(" R:pair_row_seq");
    } else if (k.p.htab) {
        k_pair_row<PR, TR, false, true><<<dim3((unsigned)k.npairs, (unsigned)(N1 / 2)), dim3(TR), 0, st>>>(k);
        plan_note(" R:pair_row_htab");
    } else if (k.p.tail_a) {
        k_pair_row<PR, TR, true><<<dim3((unsigned)k.npairs, (unsigned)(N1 / 2)), dim3(TR), 0, st>>>(k);
        plan_note(" R:pair_row_tail");
    } else if constexpr (N2 == 8192) {
        constexpr int TS = N2 / 16;                  // 16 values of each row per thread
        using PRS = PairRowsSeq<N2, TS, RF, RI>;
        k_pair_row_seq<PRS, TS, false><<<dim3((unsigned)k.npairs, (unsigned)(N1 / 2 - 1)), dim3(TS), 0, st>>>(k);
        k_pair_row_seq<PRS, TS, true><<<dim3((unsigned)k.npairs, 1u), dim3(TS), 0, st>>>(k);
        plan_note(" R:pair_row_seq");
    } else {
        k_pair_row<PR, TR><<<dim3((unsigned)k.npairs, (unsigned)(N1 / 2)), dim3(TR), 0, st>>>(k);
        plan_note(" R:pair_row");
    }
    tk_end(st);
    LAUNCHCHK();
    const bool fast = PCC::kItemsExact && fast_epilogue(k);
    // the generic pass C reads the null decisions as bits
    if (k.mask_ready && !fast) HIPCHK(hipStreamWaitEvent(st, k.mask_ready, 0));
    tk_begin(TK_COLC, st);
    if (fast) {
        if constexpr (PCC::kItemsExact) {
            if constexpr (N1 == 2048 && N2 % 16 == 0) {
                k_pairC_fast32<PairCols<N1, 16, 512, CF, CI, -1>, 512>
                    <<<dim3((unsigned)(N2 / 16), (unsigned)k.npairs), dim3(512), 0, st>>>(k);
                plan_note(" C:fast32");
            } else {
                k_pairC_fast<PCC, TC><<<dim3((unsigned)(N2 / BC), (unsigned)k.npairs), dim3(TC), 0, st>>>(k);
                plan_note(" C:fast");
            }
        }
    } else if (PC::kRegCols && fold_epilogue(k)) {
        if constexpr (PC::kRegCols) {
            // 128 columns per workgroup: the lane-private LDS staging of the
            // column (N1 x 8 B per lane) then allows ~5 workgroups per CU
            constexpr int FB = B > 128 ? 128 : B;
            using PCF = PairCols<N1, FB, FB, CF, CI>;
            k_pairC_fold<PCF, FB><<<dim3((unsigned)(N2 / FB), (unsigned)k.npairs), dim3(FB), 0, st>>>(k);
            plan_note(" C:fold");
        }
    } else {
        k_pairC<PC, T><<<gc, dim3(T), 0, st>>>(k);
        plan_note(" C:generic");
    }
    tk_end(st);
    LAUNCHCHK();
    if (fast && k.mtab) {
        if (k.mask_ready) HIPCHK(hipStreamWaitEvent(st, k.mask_ready, 0));
        const int rc = launch_null_fix(k, st);
        if (rc) return rc;
        plan_note(" N:fix_list");
    }
    return PSS_OK;
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
