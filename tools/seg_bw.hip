// Segment-width microbenchmark (diagnostic, tools/seg_bw.hip): HBM bandwidth
// of the column passes' access pattern as a function of the row-segment width.
// A workgroup owns S bytes of every one of R rows (row stride `rs` bytes) of
// two "channel" buffers -- the fast pass C's output (S = 4 B x columns, R =
// N1 rows 16 KB apart per channel) -- and writes (or reads) them; the grid
// walks the column blocks with the pipeline's XCD-aware order (xcd_block).
// Compared with the same bytes written contiguously per workgroup.
//   build: hipcc --offload-arch=gfx950 -O3 -o tools/seg_bw tools/seg_bw.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ void xcd_map(uint32_t &bx, uint32_t &by) {
    const uint32_t gx = gridDim.x, total = gx * gridDim.y;
    const uint32_t id = blockIdx.x + blockIdx.y * gx;
    const uint32_t l = ((total & 7u) == 0u) ? (id & 7u) * (total >> 3) + (id >> 3) : id;
    by = l / gx;
    bx = l - by * gx;
}

// blockIdx -> (column block bx, channel pair by); S / 16 lanes per row segment
template <int S>
__global__ __launch_bounds__(256) void k_wseg(float4 *a, float4 *b, int rows, size_t rs, size_t cs) {
    uint32_t bx, by;
    xcd_map(bx, by);
    constexpr int LPR = S / 16;                       // lanes per row segment
    const int lane = threadIdx.x % LPR, r0 = threadIdx.x / LPR;
    const float v = (float)threadIdx.x;
    char *pa = (char *)a + (size_t)(2 * by) * cs + (size_t)bx * S + lane * 16;
    char *pb = (char *)b + (size_t)(2 * by + 1) * cs + (size_t)bx * S + lane * 16;
    for (int r = r0; r < rows; r += 256 / LPR) {
        *(float4 *)(pa + (size_t)r * rs) = make_float4(v, v, v, v);
        *(float4 *)(pb + (size_t)r * rs) = make_float4(v, v, v, v);
    }
}
// the same bytes per workgroup, contiguous
template <int S>
__global__ __launch_bounds__(256) void k_wcontig(float4 *a, float4 *b, int rows, size_t rs, size_t cs) {
    uint32_t bx, by;
    xcd_map(bx, by);
    const size_t per = (size_t)rows * S;            // bytes per channel per block
    char *pa = (char *)a + (size_t)(2 * by) * cs + (size_t)bx * per;
    char *pb = (char *)b + (size_t)(2 * by + 1) * cs + (size_t)bx * per;
    const float v = (float)threadIdx.x;
    for (size_t o = threadIdx.x * 16; o < per; o += 256 * 16) {
        *(float4 *)(pa + o) = make_float4(v, v, v, v);
        *(float4 *)(pb + o) = make_float4(v, v, v, v);
    }
}
template <int S>
__global__ __launch_bounds__(256) void k_rseg(const float4 *a, float *sink, int rows, size_t rs, size_t cs) {
    uint32_t bx, by;
    xcd_map(bx, by);
    constexpr int LPR = S / 16;
    const int lane = threadIdx.x % LPR, r0 = threadIdx.x / LPR;
    const char *pa = (const char *)a + (size_t)by * cs + (size_t)bx * S + lane * 16;
    float acc = 0.f;
    for (int r = r0; r < rows; r += 256 / LPR) {
        const float4 q = *(const float4 *)(pa + (size_t)r * rs);
        acc += q.x + q.y + q.z + q.w;
    }
    if (acc == 12345.f) sink[threadIdx.x] = acc;
}
template <int S>
__global__ __launch_bounds__(256) void k_rcontig(const float4 *a, float *sink, int rows, size_t rs, size_t cs) {
    uint32_t bx, by;
    xcd_map(bx, by);
    const size_t per = (size_t)rows * S;
    const char *pa = (const char *)a + (size_t)by * cs + (size_t)bx * per;
    float acc = 0.f;
    for (size_t o = threadIdx.x * 16; o < per; o += 256 * 16) {
        const float4 q = *(const float4 *)(pa + o);
        acc += q.x + q.y + q.z + q.w;
    }
    if (acc == 12345.f) sink[threadIdx.x] = acc;
}

template <typename F>
static float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

template <int S>
static void run(float4 *buf, float *sink, int nch, int rows, size_t rs) {
    // output-like: nch channel rows of rows * rs bytes, written by pairs
    const size_t cs = (size_t)rows * rs;
    const size_t bytes = (size_t)nch * rows * (rs < (size_t)S ? rs : 0);   // (unused)
    (void)bytes;
    const int nb = (int)(rs / S);
    dim3 g(nb, nch / 2);
    const double tot = (double)nch * rows * rs;
    float t1 = timeit([&] { k_wseg<S><<<g, 256>>>(buf, buf, rows, rs, cs); }, 5);
    float t2 = timeit([&] { k_wcontig<S><<<g, 256>>>(buf, buf, rows, rs, cs); }, 5);
    dim3 gr(nb, nch);
    float t3 = timeit([&] { k_rseg<S><<<gr, 256>>>(buf, sink, rows, rs, cs); }, 5);
    float t4 = timeit([&] { k_rcontig<S><<<gr, 256>>>(buf, sink, rows, rs, cs); }, 5);
    printf("S=%4d B rows=%d stride=%zu KB: write seg %.3f ms (%.0f GB/s)  contig %.3f ms (%.0f GB/s) | "
           "read seg %.3f ms (%.0f GB/s)  contig %.3f ms (%.0f GB/s)\n",
           S, rows, rs / 1024, t1, tot / t1 / 1e6, t2, tot / t2 / 1e6, t3, tot / t3 / 1e6, t4, tot / t4 / 1e6);
}

int main(int argc, char **argv) {
    const int nch = argc > 1 ? atoi(argv[1]) : 512;
    // C3 output geometry: N = 2^22 fp32 per channel = 1024 rows of 16 KB
    const int rows = 1024;
    const size_t rs = 16384;
    const size_t total = (size_t)nch * rows * rs;
    float4 *buf;
    float *sink;
    CK(hipMalloc(&buf, total));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(buf, 0, total));
    printf("buffer %.2f GB, %d channels\n", total / 1e9, nch);
    run<32>(buf, sink, nch, rows, rs);
    run<64>(buf, sink, nch, rows, rs);
    run<128>(buf, sink, nch, rows, rs);
    run<256>(buf, sink, nch, rows, rs);
    run<512>(buf, sink, nch, rows, rs);
    // spill-like: rows of 32 KB (4096 complex), segments of 128 / 256 B
    run<128>(buf, sink, nch / 2, rows, 2 * rs);
    run<256>(buf, sink, nch / 2, rows, 2 * rs);
    CK(hipFree(buf));
    return 0;
}
