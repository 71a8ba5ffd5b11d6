// pss_fourstep.hip -- the power-of-two four-step: the dispatch, C3's 2^22 (other
// lengths: pss_fourstep_b.hip), the delayed-null mask-table kernels and fix-up.
#include "pss_engine.hpp"
#include <algorithm>

using namespace pss;

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
        // the position's coefficients, compacted; k_mask_roots turns them
        // into its root record (the scan's cost is per f-dependent position:
        // run here, every wave holding one such position would run it for
        // all 64 lanes)
        const uint32_t idx = b0 + (uint32_t)__popcll(ab & ((1ull << lane) - 1ull));
        float4 *dst = reinterpret_cast<float4 *>(coef + (int64_t)idx * KREC);
        dst[1] = make_float4(c[0], c[1], c[2], c[3]);
        dst[2] = make_float4(c[4], c[5], c[6], c[7]);
        dst[3] = make_float4(c[8], c[9], c[10], c[11]);
    }
}

// Root records of the f-dependent positions (compacted by k_mask_table, which
// left each one's Chebyshev coefficients in its record): where the fp32
// Clenshaw value crosses 1, on a certified scan grid (see root_hit).  One
// position per lane, grid-stride over the device-side count: the same
// arithmetic as the scan had inside k_mask_table, bitwise the same records.
__global__ __launch_bounds__(256) void k_mask_roots(float *coef, const uint32_t *counter) {
    const uint32_t na = *counter;
    for (uint32_t idx = blockIdx.x * 256u + threadIdx.x; idx < na; idx += gridDim.x * 256u) {
        float4 *dst = reinterpret_cast<float4 *>(coef + (int64_t)idx * KREC);
        const float4 q[3] = {dst[1], dst[2], dst[3]};
        const float c[KCH] = {q[0].x, q[0].y, q[0].z, q[0].w, q[1].x, q[1].y, q[1].z, q[1].w,
                              q[2].x, q[2].y, q[2].z, q[2].w};
        float S = 0.f;
#pragma unroll
        for (int n = 1; n < KCH; ++n) S += fabsf(c[n]);
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
        // the scan records the cells [t_{jg-1}, t_jg] where the decision flips
        // (grid points -1 + jg H are exact); the bisections run afterwards,
        // flip i of every lane together, so a wave pays 24 evaluations per
        // flip of its busiest lane rather than per flip of every lane (the
        // same brackets and evaluations: bitwise the same roots)
        int jf[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) jf[i] = 0;
        for (int jg = 1; jg <= NG; ++jg) {
            const float tg = -1.0f + (float)jg * H;
            const float g = cheb_eval_r(q, tg) - 1.0f;
            const bool cur = g > 0.0f;
            if (cur != prev) {
                cert = cert && (fabsf(g - gprev) - 2.0f * err > D2 * H * H);   // one flip only
#pragma unroll
                for (int i = 0; i < 10; ++i) if (i == cnt) jf[i] = jg;
                ++cnt;
            } else {
                // no flip: g stays within D2 H^2 / 8 of the chord between the
                // cell's ends, whose values share a sign
                cert = cert && (fminf(fabsf(g), fabsf(gprev)) - err > D2 * H * H * 0.125f);
            }
            prev = cur;
            gprev = g;
        }
        const int nb = cnt < 10 ? cnt : 10;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            if (i < nb) {
                // the decisions alternate from s0: before flip i it is s0 for even i
                const bool pv = (i & 1) ? !s0 : s0;
                float lo = -1.0f + (float)(jf[i] - 1) * H, hi = -1.0f + (float)jf[i] * H;
                for (int it = 0; it < 24; ++it) {
                    const float mid = 0.5f * (lo + hi);
                    if ((cheb_eval_r(q, mid) > 1.0f) == pv) lo = mid; else hi = mid;
                }
                rt[i] = lo;
            }
        }
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

int launch_node_params(uint64_t *ramp, float *nyq, int L, hipStream_t st) {
    k_node_params<<<1, 64, 0, st>>>(ramp, nyq, L);
    LAUNCHCHK();
    return PSS_OK;
}
int launch_mask_table(const float *nodes, int64_t N, uint2 *bits, uint32_t *base, float *coef, uint32_t *counter,
                      hipStream_t st) {
    k_mask_table<<<dim3((unsigned)(N / 256)), dim3(256), 0, st>>>(nodes, N, bits, base, coef, counter);
    LAUNCHCHK();
    const unsigned gr = (unsigned)std::min<int64_t>(N / 256, 1024);
    k_mask_roots<<<dim3(gr), dim3(256), 0, st>>>(coef, counter);
    LAUNCHCHK();
    return PSS_OK;
}
int launch_mask_words(const uint2 *bits, uint32_t nwords, uint32_t *list, uint32_t *count, hipStream_t st) {
    k_mask_words<<<dim3((nwords + 255) / 256), dim3(256), 0, st>>>(bits, nwords, list, count);
    LAUNCHCHK();
    return PSS_OK;
}
int launch_mask_bits(const KP &k, uint32_t *bm, hipStream_t st) {
    k_mask_bits<<<dim3((unsigned)((k.N / 32 + 255) / 256), (unsigned)k.p.nchan), dim3(256), 0, st>>>(k, bm);
    LAUNCHCHK();
    return PSS_OK;
}
int launch_null_fix(const KP &k, hipStream_t st) {
    tk_begin(TK_NULLFIX, st);
    // grid-stride over the word list: ~1/8 of the words per channel
    const unsigned gx = (unsigned)((k.N / 32 / 8 + 255) / 256);
    k_null_fix_list<<<dim3(gx ? gx : 1, (unsigned)k.p.nchan), dim3(256), 0, st>>>(k);
    tk_end(st);
    LAUNCHCHK();
    return PSS_OK;
}

int run_fourstep(KP &k, hipStream_t st, const float *mask_row) {
    const int64_t N = k.N;
    plan_note("fourstep");
    if (N == (1 << 22)) {
        // C3: 1024 x 4096 (two 4096-point rows of a pair in 66 KB: two row
        // workgroups per CU; 16-column pass-C blocks, 64-B output segments)
        k.N2 = 4096;
        k.N1 = 1024;
        return launch_pair<1024, 8, 512, C1kF, C1kF, 4096, 512, C4k, C4k, 256, kBC, kTC>(k, st, mask_row);
    }
    return run_fourstep_b(k, st, mask_row);
}
