// pss_device.hpp -- gfx950 device helpers: complex arithmetic, revolution-based
// native trig, fixed-point phases, Philox4x32-7 and chi-square samplers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Debug builds (PSS_DEBUG=1, tools/debug_gpu.sh): device-side bounds asserts
// on the generic-pointer accesses and on the offsets of buffer (SRD) accesses
// -- the hardware drops an out-of-range buffer store and returns 0 for an
// out-of-range load silently, so a wrong offset would otherwise go unseen.
#ifndef PSS_DEBUG
#define PSS_DEBUG 0
#endif
#if PSS_DEBUG
#include <cassert>
#define PSS_DASSERT(c) assert(c)
#else
#define PSS_DASSERT(c) ((void)0)
#endif

namespace pss {

typedef float2 cf;

// Explicit fused forms: with free contraction the compiler picks which product
// to fuse per call site, so the same math rounds differently in different
// kernels (the fast-path kernels must match the generic ones bit for bit).
__device__ __forceinline__ cf cmul(cf a, cf b) {
    return make_float2(fmaf(a.x, b.x, -(a.y * b.y)), fmaf(a.x, b.y, a.y * b.x));
}
// a * conj(b), the same fused form
__device__ __forceinline__ cf cmul_conj(cf a, cf b) {
    return make_float2(fmaf(a.x, b.x, a.y * b.y), fmaf(a.y, b.x, -(a.x * b.y)));
}
__device__ __forceinline__ cf cadd(cf a, cf b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ cf csub(cf a, cf b) { return make_float2(a.x - b.x, a.y - b.y); }

// exp(2 pi i * r) for r in revolutions, via the native gfx950 v_sin_f32 /
// v_cos_f32 (input in revolutions; measured max abs error 1.2e-7 on MI355X,
// tools/probe_trig.hip).  |r| <= 0.5 keeps the argument's own rounding small.
__device__ __forceinline__ cf expi_rev(float r) {
    return make_float2(__builtin_amdgcn_cosf(r), __builtin_amdgcn_sinf(r));
}

// 2^-64-cycle fixed point phase -> signed revolutions in [-0.5, 0.5).
__device__ __forceinline__ float fix_to_rev(uint64_t ph) {
    int32_t hi = (int32_t)(uint32_t)(ph >> 32);   // top 32 bits, signed
    return (float)hi * 2.3283064365386963e-10f;   // * 2^-32
}

// 2^-32-cycle fixed point phase -> signed revolutions in [-0.5, 0.5).
__device__ __forceinline__ float fix32_to_rev(uint32_t ph) {
    return (float)(int32_t)ph * 2.3283064365386963e-10f;   // * 2^-32
}

// --------------------------------------------------------------------------
// Buffer (SRD) access: 32-bit per-lane byte offsets plus a scalar offset, so a
// run of strided accesses costs no per-access 64-bit address VGPRs.  The base
// must be wave-uniform (kernel arguments / blockIdx only).
// --------------------------------------------------------------------------
struct Buf {
    __amdgpu_buffer_rsrc_t r;
#if PSS_DEBUG
    uint32_t nbytes;
    __device__ __forceinline__ Buf(const void *base, uint32_t bytes)
        : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000)), nbytes(bytes) {}
#define PSS_BUF_CHECK(voff, soff, w) PSS_DASSERT((uint64_t)(voff) + (soff) + (w) <= nbytes)
#else
    __device__ __forceinline__ Buf(const void *base, uint32_t bytes)
        : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000)) {}
#define PSS_BUF_CHECK(voff, soff, w) ((void)0)
#endif
    __device__ __forceinline__ cf ld2(uint32_t voff, uint32_t soff) const {
        typedef unsigned int u2 __attribute__((ext_vector_type(2)));
        PSS_BUF_CHECK(voff, soff, 8);
        u2 w = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
        return make_float2(__uint_as_float(w.x), __uint_as_float(w.y));
    }
    __device__ __forceinline__ void st2(cf v, uint32_t voff, uint32_t soff) const {
        typedef unsigned int u2 __attribute__((ext_vector_type(2)));
        PSS_BUF_CHECK(voff, soff, 8);
        u2 w;
        w.x = __float_as_uint(v.x);
        w.y = __float_as_uint(v.y);
        __builtin_amdgcn_raw_buffer_store_b64(w, r, voff, soff, 0);
    }
    // AUX = cache policy bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
    template <int AUX = 0>
    __device__ __forceinline__ float4 ld4(uint32_t voff, uint32_t soff) const {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        PSS_BUF_CHECK(voff, soff, 16);
        u4 w = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, AUX);
        return make_float4(__uint_as_float(w.x), __uint_as_float(w.y), __uint_as_float(w.z), __uint_as_float(w.w));
    }
    template <int AUX = 0>
    __device__ __forceinline__ void st4(float a, float b, float c, float d, uint32_t voff, uint32_t soff) const {
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        u4 w;
        w.x = __float_as_uint(a);
        w.y = __float_as_uint(b);
        w.z = __float_as_uint(c);
        w.w = __float_as_uint(d);
        PSS_BUF_CHECK(voff, soff, 16);
        __builtin_amdgcn_raw_buffer_store_b128(w, r, voff, soff, AUX);
    }
};

// --------------------------------------------------------------------------
// Philox4x32-7 (Salmon et al., SC'11, "Parallel random numbers: as easy as
// 1, 2, 3"): Philox4x32 with 7 rounds is the fewest their paper reports as
// passing TestU01's BigCrush (Table 2); Random123 defaults to 10 as a safety
// margin.  The step is issue-bound and power-throttled, and the 3 rounds (12
// VALU per 4 draws) are worth 0.9 ms at C3.  This is part of the stream
// definition: changing kPhiloxRounds changes every draw (DESIGN.md section 4
// and INTEGRATION.md record it); the distribution gates (KS / moments,
// tests/test_gpu_stats.py) and tools/philox_model.py's 400-seed study
// (profiles/r03/philox_quality.txt) guard the generator.
// --------------------------------------------------------------------------
static constexpr int kPhiloxRounds = 7;
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < kPhiloxRounds; ++r) {
        // one v_mad_u64_u32 per product (hi and lo together), not mul_hi + mul_lo
        const uint64_t p0 = (uint64_t)c.x * 0xD2511F53u;
        const uint64_t p1 = (uint64_t)c.z * 0xCD9E8D57u;
        // three-way xors as one v_bitop3_b32 each (truth table 0x96 = a ^ b ^ c)
        c = make_uint4(__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
                       __builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// Purposes (distinct Philox streams per stage).
enum : uint32_t { P_PULSE = 1, P_BOX = 2, P_REP = 3, P_NOISE = 4, P_TEST = 5 };

struct Rng {
    uint32_t k0, k1, word;   // key + (call_id << 4 | purpose)
    __device__ Rng(uint64_t seed, uint32_t call_id, uint32_t purpose)
        : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), word((call_id << 4) | purpose) {}
    // 4 x 32 random bits for (stream position a, b) with a 32-bit attempt tag.
    __device__ __forceinline__ uint4 bits(uint32_t a, uint32_t b, uint32_t tag) const {
        return philox(make_uint4(a, tag, b, word), k0, k1);
    }
};

// uniform in (0, 1]: fine resolution near 0 where -log(u) needs it
__device__ __forceinline__ float u01(uint32_t x) {
    return fmaf((float)x, 2.3283064365386963e-10f, 1.1641532182693481e-10f);
}

// [0, 1) from the top 23 bits of x, by the exponent trick: 1.m - 1 (one
// shift-or and one subtract, both full rate; v_cvt_f32_u32 issues at half
// rate on gfx950, tools/probe_rates.hip).  Exact: 23-bit grid of [0, 1).
__device__ __forceinline__ float frac23(uint32_t x) {
    return __uint_as_float(0x3F800000u | (x >> 9)) - 1.0f;
}

// Four chi2(1) draws from one Philox block: z^2 with z Box-Muller normals,
// -2 ln(u) cos^2(2 pi v) and -2 ln(u) sin^2(2 pi v), written as
// h (1 + cos 4 pi v) and h (1 - cos 4 pi v), h = -ln u: one transcendental
// per pair instead of two (the step is issue-bound and power-throttled).  The
// angle 2v mod 1 is the top 23 bits below bit 31 of the word (4 pi v mod 2 pi
// is uniform when v is).  Where the cosine is within an ulp of -1 or 1 the
// small member of the pair is resolved to ~ulp(h) = h 6e-8 absolute
// (chi2 values below ~1e-6; the distribution gates, tests/test_gpu_stats.py,
// cover the sampler).
// `scale` multiplies the draws inside the sampler (h scale = (-ln2 scale)
// log2 u: the product with the pulse draw_norm costs no extra instruction);
// scale = 1 gives the plain chi2(1) values.
__device__ __forceinline__ float4 chi2_1x4(uint4 r, float scale = 1.0f) {
    const float kl = -0.6931471805599453f * scale;
    const float h0 = kl * __builtin_amdgcn_logf(u01(r.x));   // -ln u = -ln2 log2 u
    const float h1 = kl * __builtin_amdgcn_logf(u01(r.z));
    const float c0 = __builtin_amdgcn_cosf(frac23(r.y << 1));                 // cos(2 pi (2v mod 1))
    const float c1 = __builtin_amdgcn_cosf(frac23(r.w << 1));
    // explicit fused forms: left to the compiler, h + h c contracts or not
    // depending on the surrounding code, and the fast and generic kernels
    // would draw values an ulp apart
    return make_float4(fmaf(h0, c0, h0), fmaf(-h0, c0, h0), fmaf(h1, c1, h1), fmaf(-h1, c1, h1));
}

// Four N(0, 1) draws from one Philox block (Box-Muller pairs
// sqrt(-2 ln u) (cos 2 pi v, sin 2 pi v)): the amplitude-pulse draws.
__device__ __forceinline__ float4 normal_x4(uint4 r) {
    const float l0 = sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(r.x)));
    const float l1 = sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(r.z)));
    const float v0 = frac23(r.y);
    const float v1 = frac23(r.w);
    return make_float4(l0 * __builtin_amdgcn_cosf(v0), l0 * __builtin_amdgcn_sinf(v0),
                       l1 * __builtin_amdgcn_cosf(v1), l1 * __builtin_amdgcn_sinf(v1));
}

// log1p(y) - y for |y| small, without cancellation (alternating series).
__device__ __forceinline__ float log1p_minus(float y) {
    if (fabsf(y) < 0.125f) {
        const float y2 = y * y;
        // -y^2/2 + y^3/3 - y^4/4 + ... (terms to y^10: error < 1e-10 for |y| < 1/8)
        float s = -1.0f / 10;
        s = fmaf(s, y, 1.0f / 9);
        s = fmaf(s, y, -1.0f / 8);
        s = fmaf(s, y, 1.0f / 7);
        s = fmaf(s, y, -1.0f / 6);
        s = fmaf(s, y, 1.0f / 5);
        s = fmaf(s, y, -1.0f / 4);
        s = fmaf(s, y, 1.0f / 3);
        s = fmaf(s, y, -0.5f);
        return s * y2;
    }
    return log1pf(y) - y;
}

// chi2(df) for general df > 0 = 2 * Gamma(df/2) via Marsaglia-Tsang (2000);
// shape < 1 boosted by U^(1/a).  One attempt: z ~ N(0, 1), y = c z, v = (1 +
// y)^3; accepted by the squeeze u < 1 - 0.0331 z^4 (no logarithm: ~all
// attempts at the large df of fold mode, Nfold ~ 1e4) or else by ln u < z^2/2
// + d (1 - v + ln v), evaluated in the cancellation-free form
// d (3 (log1p(y) - y) - 3 y^2 - y^3) so fp32 is exact enough even at
// df ~ 1e4 (d ~ 5e3, the bracket O(1/d)).
struct MtParams {
    float d, c, shape;
    bool boost;
};
__device__ __forceinline__ MtParams mt_params(float df) {
    MtParams q;
    q.shape = 0.5f * df;
    q.boost = q.shape < 1.0f;
    q.d = (q.boost ? q.shape + 1.0f : q.shape) - (1.0f / 3.0f);
    q.c = rsqrtf(9.0f * q.d);
    return q;
}
__device__ __forceinline__ bool mt_try(float z, float u, const MtParams &q, float &x) {
    const float y = q.c * z;
    if (y <= -1.0f) return false;
    const float v = (1.0f + y) * (1.0f + y) * (1.0f + y);
    const float z2 = z * z;
    if (u < fmaf(-0.0331f * z2, z2, 1.0f) ||
        0.6931471805599453f * __builtin_amdgcn_logf(u) <
            fmaf(0.5f, z2, q.d * (3.0f * log1p_minus(y) - y * y * (3.0f + y)))) {
        x = q.d * v;
        return true;
    }
    return false;
}
// Retries of sample h of a pair (rare): its own Philox block per attempt,
// tags (h + 1) << 16 | t (attempt 0 is the pair's shared block, tag 1).
__device__ __noinline__ float mt_retry(const Rng &g, uint32_t m, uint32_t b, uint32_t h, const MtParams &q) {
    float x = q.d;
    for (uint32_t t = 1; t < 64; ++t) {
        const uint4 r = g.bits(m, b, ((h + 1u) << 16) | t);
        const float z = sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(r.x))) *
                        __builtin_amdgcn_cosf(frac23(r.y));
        if (mt_try(z, u01(r.z), q, x)) break;
    }
    return x;
}
// chi2(df) draws of the PAIR of samples (2m, 2m + 1) of stream position b:
// attempt 0 of both comes from ONE Philox block -- the two Box-Muller normals
// of (r.x, r.y), the uniforms r.z and r.w -- so a sample costs half a block,
// half a logarithm and one sin or cos on the common path (fold-mode C4 draws
// every sample this way).  Keyed (m, b, attempt): results do not depend on
// how samples are grouped into launches.
__device__ __forceinline__ void chi2_pair(const Rng &g, uint32_t m, uint32_t b, float df, float &x0, float &x1) {
    const MtParams q = mt_params(df);
    const uint4 r = g.bits(m, b, 1u);
    const float sl = sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u01(r.x)));
    const float v = frac23(r.y);
    const float z0 = sl * __builtin_amdgcn_cosf(v), z1 = sl * __builtin_amdgcn_sinf(v);
    if (!mt_try(z0, u01(r.z), q, x0)) x0 = mt_retry(g, m, b, 0u, q);
    if (!mt_try(z1, u01(r.w), q, x1)) x1 = mt_retry(g, m, b, 1u, q);
    if (q.boost) {
        const uint4 ub = g.bits(m, b, 0xFFFF0000u);
        x0 *= __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(u01(ub.x)) / q.shape);
        x1 *= __builtin_amdgcn_exp2f(__builtin_amdgcn_logf(u01(ub.y)) / q.shape);
    }
    x0 *= 2.0f;
    x1 *= 2.0f;
}

// One chi2(df) draw keyed (a, b): df == 1 -> the first z^2 of block (a, b, 0);
// otherwise sample a of the pair sampler (pair a >> 1, half a & 1).
__device__ __forceinline__ float chi2_general(const Rng &g, uint32_t a, uint32_t b, float df) {
    if (df == 1.0f) {
        float4 q = chi2_1x4(g.bits(a, b, 0));
        return q.x;
    }
    float x0, x1;
    chi2_pair(g, a >> 1, b, df, x0, x1);
    return (a & 1u) ? x1 : x0;
}

}  // namespace pss
