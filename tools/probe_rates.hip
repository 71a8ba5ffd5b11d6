// probe_rates.hip -- issue cost of the VALU instructions the pipeline leans on
// (Philox multiplies, trig, log, packed fp32), measured on the device.
// Each kernel runs 8 independent dependency chains of one instruction per
// thread, 1024 iterations, on every CU; reports cycles per wave-instruction
// per SIMD (4 = full rate for wave64).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 1024
#define CHAINS 8

#define K(NAME, DECL, BODY, OUT)                                              \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) { \
        DECL;                                                                  \
        for (int it = 0; it < ITERS; ++it) {                                   \
            _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) { BODY; }       \
        }                                                                      \
        OUT;                                                                   \
    }

K(k_mul_lo, uint32_t a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = seed + threadIdx.x + c,
  asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(seed)),
  uint32_t s = 0; for (int c = 0; c < CHAINS; ++c) s ^= a[c]; out[blockIdx.x * 256 + threadIdx.x] = s)
K(k_mul_hi, uint32_t a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = seed + threadIdx.x + c,
  asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(seed)),
  uint32_t s = 0; for (int c = 0; c < CHAINS; ++c) s ^= a[c]; out[blockIdx.x * 256 + threadIdx.x] = s)
K(k_mad64, uint64_t a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = seed + threadIdx.x + c,
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(a[c]) : "v"((uint32_t)a[c]), "v"(seed) : "s0", "s1"),
  uint32_t s = 0; for (int c = 0; c < CHAINS; ++c) s ^= (uint32_t)a[c]; out[blockIdx.x * 256 + threadIdx.x] = s)
K(k_mul24, uint32_t a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = seed + threadIdx.x + c,
  asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(seed)),
  uint32_t s = 0; for (int c = 0; c < CHAINS; ++c) s ^= a[c]; out[blockIdx.x * 256 + threadIdx.x] = s)
K(k_xor, uint32_t a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = seed + threadIdx.x + c,
  asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[c]) : "v"(seed)),
  uint32_t s = 0; for (int c = 0; c < CHAINS; ++c) s ^= a[c]; out[blockIdx.x * 256 + threadIdx.x] = s)
K(k_fma, float a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = (float)(seed + threadIdx.x + c),
  asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[c]) : "v"((float)seed)),
  float s = 0; for (int c = 0; c < CHAINS; ++c) s += a[c]; out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)s)
K(k_pkfma, float2 a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = make_float2(seed + threadIdx.x + c, c),
  asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a[c]) : "v"(make_float2(seed, seed))),
  float s = 0; for (int c = 0; c < CHAINS; ++c) s += a[c].x + a[c].y; out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)s)
K(k_sin, float a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = (float)(seed + threadIdx.x + c) * 1e-3f,
  asm volatile("v_sin_f32 %0, %0" : "+v"(a[c])),
  float s = 0; for (int c = 0; c < CHAINS; ++c) s += a[c]; out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)s)
K(k_log, float a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = (float)(seed + threadIdx.x + c) + 2.f,
  asm volatile("v_log_f32 %0, %0" : "+v"(a[c])),
  float s = 0; for (int c = 0; c < CHAINS; ++c) s += a[c]; out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)s)
K(k_cvt, float a[CHAINS]; for (int c = 0; c < CHAINS; ++c) a[c] = (float)(seed + threadIdx.x + c),
  asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a[c])),
  float s = 0; for (int c = 0; c < CHAINS; ++c) s += a[c]; out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)s)

typedef void (*KF)(uint32_t *, uint32_t);

int main() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    const double clk = prop.clockRate * 1e3;   // Hz
    const int blocks = cus * 8;                 // 8 x 256 threads = 32 waves per CU
    uint32_t *out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    struct { const char *n; KF f; } ks[] = {
        {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi}, {"v_mad_u64_u32", k_mad64},
        {"v_mul_u32_u24", k_mul24}, {"v_xor_b32", k_xor}, {"v_fma_f32", k_fma},
        {"v_pk_fma_f32", k_pkfma}, {"v_sin_f32", k_sin}, {"v_log_f32", k_log},
        {"v_cvt_f32_u32", k_cvt}};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("CUs %d, clock %.0f MHz\n", cus, clk / 1e6);
    for (auto &k : ks) {
        k.f<<<blocks, 256>>>(out, 3);
        hipEventRecord(a);
        for (int r = 0; r < 5; ++r) k.f<<<blocks, 256>>>(out, 3);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double winstr = (double)blocks * 4 /*waves*/ * ITERS * CHAINS * 5;
        const double per_simd = winstr / (cus * 4.0);
        const double cyc = ms * 1e-3 * clk / per_simd;
        printf("%-16s %.2f cycles per wave-instruction per SIMD (at the nominal clock)\n", k.n, cyc);
    }
    hipFree(out);
    return 0;
}
