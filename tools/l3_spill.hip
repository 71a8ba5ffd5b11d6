// Infinity-Cache spill microbenchmark (diagnostic, tools/l3_spill.hip; VERDICT
// r04 item 2): can the four-step spill live in the 256-MiB Infinity Cache?
//
// The C3 run moves 16 of its 20.4 B per channel-sample through the spill:
// pass A writes it, the row pass reads and rewrites it, pass C reads it and
// streams the output out.  Here the same three dependent kernels run over a
// spill buffer of W MB, batch after batch, each batch's output going to a new
// slice of a large output buffer (so the output stream competes for the
// cache exactly as pass C's would):
//     k_write (W stored)  ->  k_rw (W loaded, W stored in place)
//                         ->  k_out (W loaded, W stored to the output stream)
// Reported per W: ns per spill byte for each kernel class (HIP events around
// every launch) and for the whole chain (events around the batch loop, i.e.
// launch gaps included), against the same chain at W = 4 GB (HBM).
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/l3_spill tools/l3_spill.hip
//   run:   tools/l3_spill [total_GB_per_W]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

static constexpr int kT = 256, kU = 4;   // threads per block, float4 per thread

__global__ __launch_bounds__(kT) void k_write(float4 *ws, size_t n4, float s) {
    const size_t base = (size_t)blockIdx.x * kT * kU + threadIdx.x;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const size_t i = base + (size_t)u * kT;
        if (i < n4) {
            const float v = (float)i * s;
            ws[i] = make_float4(v, v + 1.f, v + 2.f, v + 3.f);
        }
    }
}
__global__ __launch_bounds__(kT) void k_rw(float4 *ws, size_t n4, float s) {
    const size_t base = (size_t)blockIdx.x * kT * kU + threadIdx.x;
    float4 q[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const size_t i = base + (size_t)u * kT;
        q[u] = i < n4 ? ws[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const size_t i = base + (size_t)u * kT;
        if (i < n4) ws[i] = make_float4(q[u].y * s, q[u].x, q[u].w, q[u].z * s);
    }
}
__global__ __launch_bounds__(kT) void k_out(const float4 *ws, float4 *out, size_t n4, float s) {
    const size_t base = (size_t)blockIdx.x * kT * kU + threadIdx.x;
    float4 q[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const size_t i = base + (size_t)u * kT;
        q[u] = i < n4 ? ws[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const size_t i = base + (size_t)u * kT;
        if (i < n4) out[i] = make_float4(q[u].x + s, q[u].y, q[u].z, q[u].w);
    }
}

int main(int argc, char **argv) {
    const double total_gb = argc > 1 ? atof(argv[1]) : 8.0;
    const size_t kOut = (size_t)8 << 30;                       // output stream ring (8 GiB)
    const size_t sizes_mb[] = {8, 16, 32, 48, 64, 96, 128, 160, 192, 256, 384, 512, 1024, 4096};
    const size_t wmax = (size_t)4096 << 20;
    float4 *ws, *out;
    CK(hipMalloc(&ws, wmax));
    CK(hipMalloc(&out, kOut));
    CK(hipMemset(ws, 0, wmax));
    CK(hipMemset(out, 0, kOut));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const int kEv = 3 * 1024 + 2;
    std::vector<hipEvent_t> ev(kEv);
    for (auto &evt : ev) CK(hipEventCreate(&evt));
    printf("# W_MB batches | TB/s of bytes moved (events around every launch): write  rw(load+store)  "
           "out(load+store out) | chain TB/s (4 W bytes per batch, no events between launches)\n");
    for (size_t mb : sizes_mb) {
        const size_t W = mb << 20, n4 = W / 16;
        const int nb = (int)((total_gb * (1ull << 30)) / W) < 1 ? 1 : (int)((total_gb * (1ull << 30)) / W);
        const int nbt = nb > 1024 ? 1024 : nb;
        const unsigned grid = (unsigned)((n4 + kT * kU - 1) / (kT * kU));
        // warm-up (page tables, code objects)
        for (int b = 0; b < 2; ++b) {
            k_write<<<grid, kT, 0, st>>>(ws, n4, 1.f);
            k_rw<<<grid, kT, 0, st>>>(ws, n4, 1.f);
            k_out<<<grid, kT, 0, st>>>(ws, out, n4, 1.f);
        }
        CK(hipStreamSynchronize(st));
        // (1) the chain, events around every launch
        size_t off = 0;
        CK(hipEventRecord(ev[0], st));
        for (int b = 0; b < nbt; ++b) {
            if (off + W > kOut) off = 0;
            k_write<<<grid, kT, 0, st>>>(ws, n4, 1.f + b);
            CK(hipEventRecord(ev[3 * b + 1], st));
            k_rw<<<grid, kT, 0, st>>>(ws, n4, 1.f);
            CK(hipEventRecord(ev[3 * b + 2], st));
            k_out<<<grid, kT, 0, st>>>(ws, (float4 *)((char *)out + off), n4, 0.5f);
            CK(hipEventRecord(ev[3 * b + 3], st));
            off += W;
        }
        CK(hipStreamSynchronize(st));
        double t[3] = {0, 0, 0};
        for (int b = 0; b < nbt; ++b)
            for (int c = 0; c < 3; ++c) {
                float ms;
                CK(hipEventElapsedTime(&ms, ev[3 * b + c], ev[3 * b + c + 1]));
                t[c] += ms;
            }
        // (2) the same chain with no events between the launches
        hipEvent_t a = ev[kEv - 2], z = ev[kEv - 1];
        off = 0;
        CK(hipEventRecord(a, st));
        for (int b = 0; b < nbt; ++b) {
            if (off + W > kOut) off = 0;
            k_write<<<grid, kT, 0, st>>>(ws, n4, 1.f + b);
            k_rw<<<grid, kT, 0, st>>>(ws, n4, 1.f);
            k_out<<<grid, kT, 0, st>>>(ws, (float4 *)((char *)out + off), n4, 0.5f);
            off += W;
        }
        CK(hipEventRecord(z, st));
        CK(hipStreamSynchronize(st));
        float chain;
        CK(hipEventElapsedTime(&chain, a, z));
        const double bytes = (double)W * nbt;
        printf("%6zu %5d | %.2f %.2f %.2f | %.2f\n", mb, nbt, bytes / (t[0] * 1e-3) / 1e12,
               2.0 * bytes / (t[1] * 1e-3) / 1e12, 2.0 * bytes / (t[2] * 1e-3) / 1e12,
               4.0 * bytes / (chain * 1e-3) / 1e12);
        fflush(stdout);
    }
    // each kernel class alone, repeated on one W (residency without the
    // output stream between uses)
    printf("# alone (one kernel class repeated on one W): W_MB | TB/s of bytes moved: write  rw  out\n");
    for (size_t mb : {32, 64, 128, 192, 256, 512, 4096}) {
        const size_t W = (size_t)mb << 20, n4 = W / 16;
        const unsigned grid = (unsigned)((n4 + kT * kU - 1) / (kT * kU));
        const int reps = (int)(((size_t)8 << 30) / W) < 2 ? 2 : (int)(((size_t)8 << 30) / W);
        double r[3];
        for (int c = 0; c < 3; ++c) {
            hipEvent_t a = ev[0], z = ev[1];
            for (int w = 0; w < 2; ++w) {
                if (c == 0) k_write<<<grid, kT, 0, st>>>(ws, n4, 1.f);
                if (c == 1) k_rw<<<grid, kT, 0, st>>>(ws, n4, 1.f);
                if (c == 2) k_out<<<grid, kT, 0, st>>>(ws, out, n4, 1.f);
            }
            CK(hipEventRecord(a, st));
            for (int i = 0; i < reps; ++i) {
                if (c == 0) k_write<<<grid, kT, 0, st>>>(ws, n4, 1.f + i);
                if (c == 1) k_rw<<<grid, kT, 0, st>>>(ws, n4, 1.f);
                if (c == 2)
                    k_out<<<grid, kT, 0, st>>>(ws, (float4 *)((char *)out + (size_t)(i % (int)(kOut / W)) * W), n4,
                                               1.f);
            }
            CK(hipEventRecord(z, st));
            CK(hipStreamSynchronize(st));
            float ms;
            CK(hipEventElapsedTime(&ms, a, z));
            const double moved = (double)W * reps * (c == 0 ? 1 : 2);
            r[c] = ms * 1e6 / moved;
        }
        printf("%6zu | %.2f %.2f %.2f\n", mb, 1e-3 / r[0], 1e-3 / r[1], 1e-3 / r[2]);
        fflush(stdout);
    }
    CK(hipFree(ws));
    CK(hipFree(out));
    return 0;
}
