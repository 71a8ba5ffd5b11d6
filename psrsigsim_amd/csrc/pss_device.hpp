// pss_device.hpp -- gfx950 device helpers: complex arithmetic, revolution-based
// native trig, fixed-point phases, Philox4x32-10 and chi-square samplers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pss {

typedef float2 cf;

__device__ __forceinline__ cf cmul(cf a, cf b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
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

// --------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11)
// --------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
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
__device__ __forceinline__ double u01d(uint32_t x, uint32_t y) {
    uint64_t v = ((uint64_t)x << 21) ^ (uint64_t)(y >> 11);   // 53 bits
    return ((double)(v & ((1ull << 53) - 1)) + 0.5) * 1.1102230246251565e-16;
}

// Four chi2(1) draws from one Philox block: z^2 with z Box-Muller normals,
// -2 ln(u) cos^2(2 pi v) and -2 ln(u) sin^2(2 pi v).
__device__ __forceinline__ float4 chi2_1x4(uint4 r) {
    float l0 = -1.3862943611198906f * __builtin_amdgcn_logf(u01(r.x));   // -2 ln u = -2 ln2 log2 u
    float l1 = -1.3862943611198906f * __builtin_amdgcn_logf(u01(r.z));
    float v0 = (float)(r.y >> 8) * 5.9604644775390625e-08f;             // [0,1) revolutions
    float v1 = (float)(r.w >> 8) * 5.9604644775390625e-08f;
    float c0 = __builtin_amdgcn_cosf(v0), s0 = __builtin_amdgcn_sinf(v0);
    float c1 = __builtin_amdgcn_cosf(v1), s1 = __builtin_amdgcn_sinf(v1);
    return make_float4(l0 * c0 * c0, l0 * s0 * s0, l1 * c1 * c1, l1 * s1 * s1);
}

// chi2(df) for general df > 0 = 2 * Gamma(df/2) via Marsaglia-Tsang (2000);
// shape < 1 boosted by U^(1/a).  Double precision acceptance test (the
// d(1 - v + ln v) term cancels catastrophically in fp32 at df ~ 1e4).
// Each attempt consumes one Philox block keyed (a, b, attempt).
__device__ __noinline__ float chi2_general(const Rng &g, uint32_t a, uint32_t b, float df) {
    if (df == 1.0f) {
        float4 q = chi2_1x4(g.bits(a, b, 0));
        return q.x;
    }
    double shape = 0.5 * (double)df;
    bool boost = shape < 1.0;
    double aa = boost ? shape + 1.0 : shape;
    double d = aa - 1.0 / 3.0;
    double c = 1.0 / sqrt(9.0 * d);
    double x = d;
    for (uint32_t t = 0; t < 64; ++t) {
        uint4 r = g.bits(a, b, t + 1);
        double u1 = u01d(r.x, r.y);
        double u2 = u01d(r.z, r.w);
        // one normal from the first pair (Box-Muller), u from the rest
        uint4 r2 = g.bits(a, b, 0x8000u + t);
        double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        double v = 1.0 + c * z;
        if (v <= 0.0) continue;
        v = v * v * v;
        double u = u01d(r2.x, r2.y);
        if (log(u) < 0.5 * z * z + d - d * v + d * log(v)) {
            x = d * v;
            if (boost) x *= pow(u01d(r2.z, r2.w), 1.0 / shape);
            break;
        }
    }
    return (float)(2.0 * x);
}

}  // namespace pss
