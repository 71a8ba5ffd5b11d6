// pss_fallback.hip -- the other even lengths: direct DFT (N <= 8192), Bluestein
// chirp-z (N > 8192), the float64 null refine of the packed paths, odd-N shift_t.
#include "pss_engine.hpp"

using namespace pss;

int launch_box_row(const KP &k, float *row, hipStream_t st);   // pss_pipeline.hip

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

// The float64 mask value m(n) at sample n of channel r, ONE recurrence shared
// by the candidate-list kernel and the per-sample (overflow) kernel, so both
// make the same decisions bit for bit: lane l walks the bins k = 1 + l + 64 j
// in order with the phasor e^{2 pi i k phi} stepped by e^{2 pi i 64 phi}
// (refine_start / refine_bin), the lanes' sums are combined by the same
// xor-shuffle tree (refine_finish).
struct RefineChain {
    double sn, cs, s64, c64, acc;
};
__device__ __forceinline__ void refine_start(const KP &k, int r, int64_t ns, int lane, RefineChain &q) {
    double phi = (double)ns / (double)k.N - (double)k.p.ramp[r] * 5.421010862427522e-20;     // n/N - s (rev)
    phi -= floor(phi);
    sincospi(2.0 * phi * (double)(1 + lane), &q.sn, &q.cs);
    sincospi(2.0 * phi * 64.0, &q.s64, &q.c64);
    q.acc = 0.0;
}
__device__ __forceinline__ void refine_bin(double2 b, RefineChain &q) {
    q.acc = fma(b.x, q.cs, fma(-b.y, q.sn, q.acc));
    const double t = q.cs * q.c64 - q.sn * q.s64;
    q.sn = q.cs * q.s64 + q.sn * q.c64;
    q.cs = t;
}
__device__ __forceinline__ double refine_finish(const KP &k, const double2 *B, int r, int64_t ns, double a) {
    const int64_t N = k.N, H = N / 2;
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    double m = B[0].x + 2.0 * a;
    if (2 * H == N) m += B[H].x * (double)k.p.nyq_im[r] * ((ns & 1) ? -1.0 : 1.0);
    return m / (double)N;
}
// wave-wide (every lane of the wave calls it for the same (r, ns)), the
// result valid in every lane
__device__ __forceinline__ double refine_mask(const KP &k, const double2 *B, int r, int64_t ns, int lane) {
    const int64_t H = k.N / 2;
    RefineChain q;
    refine_start(k, r, ns, lane, q);
    for (int64_t kb = 1 + lane; kb < H; kb += 64) refine_bin(B[kb], q);
    return refine_finish(k, B, r, ns, q.acc);
}

static __device__ __forceinline__ bool refine_cand(const cf *z, int64_t n, int64_t N, float band) {
    return n < N && fabsf(z[n < N ? n : 0].y - 1.0f) < band;
}

// candidates of every row into the list (entry = r << 32 | n; order free:
// each entry's decision is computed on its own)
__global__ __launch_bounds__(256) void k_null_cands(KP k, const cf *W1, const unsigned int *mx,
                                                   unsigned long long *list, unsigned long long *cnt, int64_t cap) {
    const int r = blockIdx.y, lane = threadIdx.x & 63;
    const int64_t N = k.N;
    const float band = fmaxf(1e-3f, 3e-5f * __uint_as_float(mx[r]));
    const int64_t n = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool cand = refine_cand(W1 + (int64_t)r * N, n, N, band);
    const uint64_t m = __ballot(cand);
    if (!m) return;
    // 64-bit count: nchan x N candidates may pass 2^32 (a wrapped 32-bit
    // count would hide an overflow of the list from the per-sample kernel)
    unsigned long long b0 = 0;
    if (lane == 0) b0 = atomicAdd(cnt, (unsigned long long)__popcll(m));
    b0 = __shfl(b0, 0);
    if (cand) {
        const int64_t idx = (int64_t)b0 + __popcll(m & ((1ull << lane) - 1ull));
        if (idx < cap) list[idx] = ((unsigned long long)r << 32) | (unsigned long long)n;
    }
}

// four candidates per wave, sixteen per workgroup: the box spectrum goes
// through LDS in 1024-bin tiles that the workgroup's 16 candidates share,
// and every bin serves four phasor recurrences per wave (the candidates'
// independent chains).  Each candidate's chain is refine_mask's (the same
// bins per lane, in the same order, the same combination).
__global__ __launch_bounds__(256) void k_null_refine_list(KP k, cf *W1, const double2 *B,
                                                         const unsigned long long *list, const unsigned long long *cnt,
                                                         int64_t cap) {
    constexpr int C = 4, TB = 1024;
    __shared__ double2 tile[TB];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t total = (int64_t)min(*cnt, (unsigned long long)cap);
    const int64_t N = k.N, H = N / 2;
    for (int64_t g0 = (int64_t)blockIdx.x * 16; g0 < total; g0 += (int64_t)gridDim.x * 16) {
        const int64_t e0 = g0 + wv * C;
        int r[C];
        int64_t ns[C];
        RefineChain q[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int64_t e = e0 + c < total ? e0 + c : g0;           // (a repeat of g0: not written)
            const unsigned long long v = list[e];
            r[c] = (int)(v >> 32);
            ns[c] = (int64_t)(v & 0xffffffffull);
            refine_start(k, r[c], ns[c], lane, q[c]);
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
                for (int c = 0; c < C; ++c) refine_bin(b, q[c]);
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const double m = refine_finish(k, B, r[c], ns[c], q[c].acc);
            if (lane == 0 && e0 + c < total) W1[(int64_t)r[c] * N + ns[c]].y = m > 1.0 ? 2.0f : 0.0f;
        }
    }
}

// the per-sample form: only when the candidate list overflowed its capacity
__global__ __launch_bounds__(256) void k_null_refine(KP k, cf *W1, const double2 *B, const unsigned int *mx,
                                                    const unsigned long long *cnt, int64_t cap) {
    if (*cnt <= (unsigned long long)cap) return;
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


int launch_null_refine(KP &k, hipStream_t st) {
    const WsLayout w = ws_layout(k.p.nchan, k.N, k.p.htab != nullptr);
    char *base = reinterpret_cast<char *>(k.p.work);
    cf *W1 = reinterpret_cast<cf *>(base);
    double2 *tw = reinterpret_cast<double2 *>(base + w.rf_tw);
    double2 *B = reinterpret_cast<double2 *>(base + w.rf_B);
    unsigned int *mx = reinterpret_cast<unsigned int *>(base + w.rf_mx);
    const float *box = k.p.inj_box;
    if (!box) {
        float *row = reinterpret_cast<float *>(base + w.row);
        const int rc = launch_box_row(k, row, st);
        if (rc) return rc;
        box = row;
    }
    k_tw64<<<stream_grid(k.N, 1), dim3(256), 0, st>>>(k.N, tw);
    LAUNCHCHK();
    double2 *part = reinterpret_cast<double2 *>(base + w.rf_part);
    unsigned long long *list = reinterpret_cast<unsigned long long *>(base + w.rf_list);
    unsigned long long *cnt = reinterpret_cast<unsigned long long *>(base + w.rf_cnt);
    const int64_t K = k.N / 2 + 1, cap = (g_flags & PSS_FLAG_REFINE_PER_SAMPLE) ? 0 : refine_cap(k.p.nchan, k.N);
    k_null_bspec<<<dim3((unsigned)((K + 255) / 256), (unsigned)kBsParts), dim3(256), 0, st>>>(box, k.N, tw, part);
    LAUNCHCHK();
    k_null_bsum<<<dim3((unsigned)((K + 255) / 256)), dim3(256), 0, st>>>(part, K, B);
    LAUNCHCHK();
    HIPCHK(hipMemsetAsync(mx, 0, (size_t)k.p.nchan * 4, st));
    HIPCHK(hipMemsetAsync(cnt, 0, 8, st));
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
    plan_note(cap ? " N:refine_list" : " N:refine_per_sample");
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
    plan_note("bluestein %lldx%lld %s%s", (long long)g.M1, (long long)g.M2, pair ? "pair" : "rows",
              fused ? " fused" : "");
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

int launch_fb_epilogue(KP &k, hipStream_t st) {
    k_fb_epilogue<<<stream_grid((k.N + 3) / 4, k.p.nchan), dim3(256), 0, st>>>(k);
    LAUNCHCHK();
    return PSS_OK;
}

int run_fallback(KP &k, hipStream_t st) {
    if (bs_len(k.N) && !(g_flags & PSS_FLAG_DIRECT_DFT)) return run_bluestein(k, st);
    dim3 g = stream_grid((k.N + 3) / 4, k.p.nchan);
    plan_note("direct");
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

// odd n: forward N-point direct DFT x ramp, then the (N - 1)-point inverse
int shift_rows_odd(float *rows, int32_t nrows, int64_t n, int64_t ld, const uint64_t *ramp, void *work,
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
