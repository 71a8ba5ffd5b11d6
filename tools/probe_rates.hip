// probe_rates.hip -- issue cost of the VALU instructions the pipeline leans on
// (Philox multiplies, bit ops, trig, log, packed fp32), measured on the device
// at the IN-KERNEL clock, for 1, 2, 4 and 8 waves per SIMD.
//
// Each wave runs CHAINS independent dependency chains of one instruction,
// ITERS iterations, and stamps s_memtime (shader clock) and s_memrealtime
// (100 MHz) around the loop: in-kernel clock = median over waves of
// s_memtime delta / s_memrealtime delta * 100 MHz.  Launches of W waves per
// SIMD (256-thread blocks, one wave per SIMD each, CUs * W blocks, all
// resident): cycles per wave-instruction per SIMD =
//     wall time (hipEvents over 10 launches) * in-kernel clock
//     / (W * ITERS * CHAINS * 10).
// Stamps go to their own buffer (never an output).  Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define ITERS 16384
#define CHAINS 8

#define K(NAME, T, INIT, BODY, FOLD)                                                      \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint64_t *st, uint32_t seed) { \
        T a[CHAINS];                                                                       \
        for (int c = 0; c < CHAINS; ++c) a[c] = INIT;                                      \
        __syncthreads();                                                                   \
        const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
        for (int it = 0; it < ITERS; ++it) {                                               \
            _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) { BODY; }                   \
        }                                                                                  \
        uint32_t s = 0;                                                                    \
        for (int c = 0; c < CHAINS; ++c) s ^= FOLD;                                        \
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
        const uint32_t gw = (blockIdx.x * 256 + threadIdx.x) >> 6;                         \
        if ((threadIdx.x & 63) == 0) { st[2 * gw] = t1 - t0; st[2 * gw + 1] = r1 - r0; }   \
        out[blockIdx.x * 256 + threadIdx.x] = s;                                           \
    }

K(k_fma, float, (float)(seed + threadIdx.x + c), asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[c]) : "v"((float)seed), "v"((float)threadIdx.x)),
  (uint32_t)a[c])
K(k_fma_same, float, (float)(seed + threadIdx.x + c), asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[c]) : "v"((float)seed)),
  (uint32_t)a[c])
K(k_add, float, (float)(seed + threadIdx.x + c), asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[c]) : "v"((float)seed)),
  (uint32_t)a[c])
K(k_pkfma, float2, make_float2(seed + threadIdx.x + c, c),
  asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(make_float2(seed, seed))), (uint32_t)(a[c].x + a[c].y))
K(k_pkadd, float2, make_float2(seed + threadIdx.x + c, c),
  asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[c]) : "v"(make_float2(seed, seed))), (uint32_t)(a[c].x + a[c].y))
K(k_pkmul, float2, make_float2(seed + threadIdx.x + c, c),
  asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[c]) : "v"(make_float2(1.0f, 1.0f))), (uint32_t)(a[c].x + a[c].y))
K(k_mul, float, (float)(seed + threadIdx.x + c), asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[c]) : "v"(1.0f)),
  (uint32_t)a[c])
K(k_mul_lo, uint32_t, seed + threadIdx.x + c, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(seed)), a[c])
K(k_mul_hi, uint32_t, seed + threadIdx.x + c, asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(seed)), a[c])
K(k_mad64, uint64_t, seed + threadIdx.x + c,
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a[c]) : "v"((uint32_t)a[c]), "v"(seed) : "s0", "s1"),
  (uint32_t)a[c])
K(k_mul24, uint32_t, seed + threadIdx.x + c, asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(seed)), a[c])
K(k_mulhi24, uint32_t, seed + threadIdx.x + c, asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(seed)), a[c])
K(k_xor, uint32_t, seed + threadIdx.x + c, asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(seed)), a[c])
K(k_bitop3, uint32_t, seed + threadIdx.x + c,
  asm volatile("v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96" : "+v"(a[c]) : "v"(seed)), a[c])
K(k_sin, float, (float)(seed + threadIdx.x + c) * 1e-3f, asm volatile("v_sin_f32 %0, %0" : "+v"(a[c])), (uint32_t)a[c])
K(k_log, float, (float)(seed + threadIdx.x + c) + 2.f, asm volatile("v_log_f32 %0, %0" : "+v"(a[c])), (uint32_t)a[c])
K(k_cvt, float, (float)(seed + threadIdx.x + c), asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[c])), (uint32_t)a[c])

typedef void (*KF)(uint32_t *, uint64_t *, uint32_t);

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    printf("CUs %d, nominal clock %.0f MHz\n", cus, prop.clockRate * 1e-3);
    const int maxw = 8;
    const int maxblocks = cus * maxw;                 // 256-thread blocks: 4 waves, one per SIMD
    uint32_t *out;
    uint64_t *st;
    hipMalloc(&out, (size_t)maxblocks * 256 * 4);
    hipMalloc(&st, (size_t)maxblocks * 4 * 2 * 8);
    std::vector<uint64_t> h((size_t)maxblocks * 4 * 2);
    hipEvent_t ea, eb;
    hipEventCreate(&ea);
    hipEventCreate(&eb);
    struct { const char *n; KF f; } ks[] = {
        {"v_fma_f32", k_fma},       {"v_fma_f32 (a,s,s)", k_fma_same}, {"v_add_f32", k_add},         {"v_pk_fma_f32", k_pkfma},
        {"v_pk_add_f32", k_pkadd},  {"v_pk_mul_f32", k_pkmul},   {"v_mul_f32", k_mul},
        {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi},   {"v_mad_u64_u32", k_mad64},
        {"v_mul_u32_u24", k_mul24}, {"v_mul_hi_u32_u24", k_mulhi24}, {"v_xor_b32", k_xor},
        {"v_bitop3_b32", k_bitop3}, {"v_sin_f32", k_sin},         {"v_log_f32", k_log},
        {"v_cvt_f32_u32", k_cvt}};
    printf("%-18s", "instruction");
    for (int w = 1; w <= maxw; w *= 2) printf("  W=%d cyc (clk MHz)", w);
    printf("\n");
    for (auto &k : ks) {
        printf("%-18s", k.n);
        for (int w = 1; w <= maxw; w *= 2) {
            const int blocks = cus * w;
            k.f<<<blocks, 256>>>(out, st, 3);          // warm-up (clock ramp)
            hipEventRecord(ea);
            const int reps = 10;
            for (int r = 0; r < reps; ++r) k.f<<<blocks, 256>>>(out, st, 3);
            hipEventRecord(eb);
            hipEventSynchronize(eb);
            float ms = 0.f;
            hipEventElapsedTime(&ms, ea, eb);
            const int nw = blocks * 4;
            hipMemcpy(h.data(), st, (size_t)nw * 2 * 8, hipMemcpyDeviceToHost);
            std::vector<double> cyc(nw), clk(nw);
            for (int i = 0; i < nw; ++i) {
                cyc[i] = (double)h[2 * i] / ((double)ITERS * CHAINS * w);
                clk[i] = h[2 * i + 1] ? (double)h[2 * i] / (double)h[2 * i + 1] * 100.0 : 0.0;
            }
            std::nth_element(clk.begin(), clk.begin() + nw / 2, clk.end());
            // wall: all SIMDs busy for the whole launch; cycles per
            // wave-instruction per SIMD = time * clock / instructions per SIMD
            const double per_simd = (double)w * ITERS * CHAINS * reps;
            const double cw = ms * 1e-3 * clk[nw / 2] * 1e6 / per_simd;
            printf("  %6.2f (%6.0f)    ", cw, clk[nw / 2]);
        }
        printf("\n");
    }
    hipFree(out);
    hipFree(st);
    return 0;
}
