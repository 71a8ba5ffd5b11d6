// pss_fft.hpp -- workgroup-level batched complex FFT for gfx950.
//
// Stockham autosort formulation (natural order in, natural order out, no bit
// reversal), mixed radix, butterflies in registers, one LDS exchange between
// stages.  A workgroup of T threads transforms BATCH sequences of length L;
// every thread permanently holds E = L*BATCH/T complex values.
//
// Register mapping for a stage of radix R: value v[ib*R + q] (ib < E/R) is
// element q of butterfly j = tid + ib*T, i.e. sequence b = j / (L/R) at
// position jj + q*(L/R) with jj = j % (L/R).  On entry the first stage's
// mapping must hold the INPUT positions; on exit the last stage's mapping holds
// the OUTPUT positions (natural order).  Running the inverse with the reversed
// radix list therefore starts from exactly the registers the forward left --
// the row kernel fuses forward FFT -> ramp -> inverse FFT without touching LDS
// in between.
//
// LDS layout: sequence b at row offset b*RS; inside a row an XOR swizzle per
// aligned 16-complex block (Lds below; DESIGN.md "LDS layout").
#pragma once
#include "pss_device.hpp"

namespace pss {

// cos/sin(2 pi k / 64), k = 0..63 (exactly 0/+-1 where the angle is a
// multiple of pi/2).
__device__ constexpr float kCos64[64] = {
    1.0f, 0.99518472667219693f, 0.98078528040323043f, 0.95694033573220882f,
    0.92387953251128674f, 0.88192126434835505f, 0.83146961230254524f, 0.77301045336273699f,
    0.70710678118654757f, 0.63439328416364549f, 0.55557023301960229f, 0.47139673682599781f,
    0.38268343236508984f, 0.29028467725446233f, 0.19509032201612833f, 0.098017140329560687f,
    0.0f, -0.098017140329560576f, -0.19509032201612819f, -0.29028467725446222f,
    -0.38268343236508973f, -0.4713967368259977f, -0.55557023301960196f, -0.63439328416364538f,
    -0.70710678118654746f, -0.77301045336273699f, -0.83146961230254524f, -0.88192126434835494f,
    -0.92387953251128674f, -0.95694033573220882f, -0.98078528040323043f, -0.99518472667219682f,
    -1.0f, -0.99518472667219693f, -0.98078528040323043f, -0.95694033573220894f,
    -0.92387953251128685f, -0.88192126434835505f, -0.83146961230254546f, -0.7730104533627371f,
    -0.70710678118654768f, -0.63439328416364593f, -0.55557023301960218f, -0.47139673682599786f,
    -0.38268343236509034f, -0.29028467725446244f, -0.19509032201612866f, -0.098017140329560798f,
    0.0f, 0.098017140329560451f, 0.19509032201612803f, 0.29028467725446205f,
    0.38268343236508967f, 0.47139673682599764f, 0.55557023301960196f, 0.63439328416364527f,
    0.70710678118654746f, 0.77301045336273666f, 0.83146961230254501f, 0.88192126434835494f,
    0.92387953251128652f, 0.95694033573220882f, 0.98078528040323032f, 0.99518472667219693f};

// e^{-+2 pi i k/R} * x for compile-time-foldable k (forward uses the minus).
template <int R, bool INV>
__device__ __forceinline__ cf rot(int k, cf x) {
    if (k == 0) return x;
    if (4 * k == R) return INV ? make_float2(-x.y, x.x) : make_float2(x.y, -x.x);
    const int idx = (k * (64 / R)) & 63;
    const float c = kCos64[idx];
    const float s = kCos64[(idx + 48) & 63];          // sin(a) = cos(a - pi/2)
    const cf w = make_float2(c, INV ? s : -s);
    return cmul(x, w);
}

template <int R, bool INV>
__device__ __forceinline__ void dft(cf *a);

// -+i * x (forward multiplies by -i)
template <bool INV>
__device__ __forceinline__ cf mul_mi(cf x) { return INV ? make_float2(-x.y, x.x) : make_float2(x.y, -x.x); }

// Radix 3: y1,2 = a0 - (a1 + a2)/2 -+ i sin(2 pi/3) (a1 - a2)  (forward: -)
template <bool INV>
__device__ __forceinline__ void dft3(cf *a) {
    constexpr float S3 = 0.86602540378443865f;
    const cf t1 = cadd(a[1], a[2]);
    const cf d = csub(a[1], a[2]);
    const cf t2 = make_float2(fmaf(-0.5f, t1.x, a[0].x), fmaf(-0.5f, t1.y, a[0].y));
    const cf r = mul_mi<INV>(make_float2(S3 * d.x, S3 * d.y));
    a[0] = cadd(a[0], t1);
    a[1] = cadd(t2, r);
    a[2] = csub(t2, r);
}

// Radix 5 (conjugate-pair form): with b1 = a1 + a4, b2 = a2 + a3, d1 = a1 - a4,
// d2 = a2 - a3:  y1,4 = a0 + c1 b1 + c2 b2 -+ i (s1 d1 + s2 d2),
//                y2,3 = a0 + c2 b1 + c1 b2 -+ i (s2 d1 - s1 d2)   (forward: -)
template <bool INV>
__device__ __forceinline__ void dft5(cf *a) {
    constexpr float C1 = 0.30901699437494742f, C2 = -0.80901699437494742f;
    constexpr float S1 = 0.95105651629515357f, S2 = 0.58778525229247313f;
    const cf b1 = cadd(a[1], a[4]), b2 = cadd(a[2], a[3]);
    const cf d1 = csub(a[1], a[4]), d2 = csub(a[2], a[3]);
    const cf r1 = make_float2(fmaf(C2, b2.x, fmaf(C1, b1.x, a[0].x)), fmaf(C2, b2.y, fmaf(C1, b1.y, a[0].y)));
    const cf r2 = make_float2(fmaf(C1, b2.x, fmaf(C2, b1.x, a[0].x)), fmaf(C1, b2.y, fmaf(C2, b1.y, a[0].y)));
    const cf i1 = mul_mi<INV>(make_float2(fmaf(S2, d2.x, S1 * d1.x), fmaf(S2, d2.y, S1 * d1.y)));
    const cf i2 = mul_mi<INV>(make_float2(fmaf(-S1, d2.x, S2 * d1.x), fmaf(-S1, d2.y, S2 * d1.y)));
    a[0] = cadd(a[0], cadd(b1, b2));
    a[1] = cadd(r1, i1);
    a[4] = csub(r1, i1);
    a[2] = cadd(r2, i2);
    a[3] = csub(r2, i2);
}

// Compile-time cos / sin (double-precision series evaluated by the compiler).
constexpr double cx_pi = 3.14159265358979323846;
// cos(pi x) for x in [-1, 1] by range reduction to [-1/4, 1/4] and Taylor series
constexpr double cx_cospi_red(double x, bool sin_form) {
    const double t = cx_pi * x, t2 = t * t;
    double s = 0.0, term = sin_form ? t : 1.0;
    for (int n = 0; n < 14; ++n) {
        s += term;
        const int a = sin_form ? 2 * n + 2 : 2 * n + 1, b = a + 1;
        term *= -t2 / ((double)a * (double)b);
    }
    return s;
}
constexpr double cx_cospi(double x) {
    // x -> [0, 2), then the octant
    while (x < 0.0) x += 2.0;
    while (x >= 2.0) x -= 2.0;
    if (x > 1.0) x = 2.0 - x;                          // cos(pi x) even about 1
    if (x == 0.5) return 0.0;
    if (x == 0.0) return 1.0;
    if (x == 1.0) return -1.0;
    if (x <= 0.25) return cx_cospi_red(x, false);
    if (x <= 0.75) return cx_cospi_red(0.5 - x, true);   // cos(pi x) = sin(pi (1/2 - x))
    return -cx_cospi_red(1.0 - x, false);
}
constexpr double cx_sinpi(double x) { return cx_cospi(x - 0.5); }

// The radix-2 DIT butterfly with a compile-time twiddle w = e^{-+2 pi i K/R}
// (forward: minus): p = e + w o, m = e - w o in six fused multiply-adds
// instead of a complex product and two complex adds (eight): o w = c u with
// u = (o.x - (s/c) o.y, o.y + (s/c) o.x) when |c| >= |s| (else s u', u' =
// ((c/s) o.x - o.y, (c/s) o.y + o.x)), so the ratio folds into u and the
// scale into the adds (Linzer & Feig's FMA butterfly); w = +-1, +-i need no
// product.
template <int R, int K, bool INV>
__device__ __forceinline__ void bfly(cf e, cf o, cf &p, cf &m) {
    constexpr int k = ((K % R) + R) % R;
    if constexpr (k == 0) {
        p = cadd(e, o);
        m = csub(e, o);
    } else if constexpr (4 * k == R) {
        const cf t = INV ? make_float2(-o.y, o.x) : make_float2(o.y, -o.x);
        p = cadd(e, t);
        m = csub(e, t);
    } else {
        constexpr double cd = cx_cospi(2.0 * k / R);
        constexpr double sd = (INV ? 1.0 : -1.0) * cx_sinpi(2.0 * k / R);
        constexpr bool by_c = (cd < 0 ? -cd : cd) >= (sd < 0 ? -sd : sd);
        constexpr float sc = (float)(by_c ? cd : sd);              // the scale: c or s
        constexpr float r = (float)(by_c ? sd / cd : cd / sd);      // tan or cot
        cf u;
        if constexpr (by_c) {
            if constexpr (r == 1.0f) {
                u = make_float2(o.x - o.y, o.y + o.x);
            } else if constexpr (r == -1.0f) {
                u = make_float2(o.x + o.y, o.y - o.x);
            } else {
                u = make_float2(fmaf(-r, o.y, o.x), fmaf(r, o.x, o.y));
            }
        } else {
            u = make_float2(fmaf(r, o.x, -o.y), fmaf(r, o.y, o.x));
        }
        p = make_float2(fmaf(sc, u.x, e.x), fmaf(sc, u.y, e.y));
        m = make_float2(fmaf(-sc, u.x, e.x), fmaf(-sc, u.y, e.y));
    }
}
template <int R, int K, int H, bool INV>
__device__ __forceinline__ void bfly_all(const cf *e, const cf *o, cf *a) {
    if constexpr (K < H) {
        bfly<R, K, INV>(e[K], o[K], a[K], a[K + H]);
        bfly_all<R, K + 1, H, INV>(e, o, a);
    }
}

// In-register DFT of size R: 3 and 5 directly; powers of two by recursive
// radix-2 DIT (with full unrolling every index and twiddle is a compile-time
// constant).
template <int R, bool INV>
__device__ __forceinline__ void dft(cf *a) {
    if constexpr (R == 3) {
        dft3<INV>(a);
    } else if constexpr (R == 5) {
        dft5<INV>(a);
    } else if constexpr (R == 2) {
        cf t = a[1];
        a[1] = csub(a[0], t);
        a[0] = cadd(a[0], t);
    } else if constexpr (R > 2) {
        constexpr int H = R / 2;
        cf e[H], o[H];
#pragma unroll
        for (int i = 0; i < H; ++i) {
            e[i] = a[2 * i];
            o[i] = a[2 * i + 1];
        }
        dft<H, INV>(e);
        dft<H, INV>(o);
        bfly_all<R, 0, H, INV>(e, o, a);
    }
}

// --------------------------------------------------------------------------
// Register-resident DFT of a short mixed-radix length (the fold-mode
// four-step's columns, N1 in {6, 10, 12, 20, 24, 30, 40, 48, 60}): one thread
// holds a whole column, so the transform needs no LDS exchange at all.
// Decimation in time, N = R M (R = 4, 2, 3 or 5): the R decimated
// subsequences x[R m + r] are transformed recursively, then for every k < M
// the radix-R butterfly over r of W_N^{r k} Y_r[k] gives X[k + M q].  With
// full unrolling every twiddle is a compile-time constant (cx_cospi above:
// double-precision Taylor series evaluated by the compiler, rounded once to
// fp32; exact 0 / +-1 at multiples of pi/2).
// --------------------------------------------------------------------------

// W_N^k x = e^{-+2 pi i k / N} x with a compile-time k (forward: minus)
template <int N, int K, bool INV>
__device__ __forceinline__ cf rot_n(cf x) {
    constexpr int k = ((K % N) + N) % N;
    if constexpr (k == 0) {
        return x;
    } else if constexpr (4 * k == N) {
        return INV ? make_float2(-x.y, x.x) : make_float2(x.y, -x.x);
    } else if constexpr (2 * k == N) {
        return make_float2(-x.x, -x.y);
    } else if constexpr (4 * k == 3 * N) {
        return INV ? make_float2(x.y, -x.x) : make_float2(-x.y, x.x);
    } else {
        constexpr float c = (float)cx_cospi(2.0 * k / N);
        constexpr float s = (float)cx_sinpi(2.0 * k / N);
        return cmul(x, make_float2(c, INV ? s : -s));
    }
}

template <int N, bool INV>
struct RegDft {
    static constexpr int R = (N % 4 == 0 && N > 4) ? 4 : (N % 2 == 0) ? 2 : (N % 3 == 0) ? 3 : 5;
    static constexpr int M = N / R;
    // y[k + M q] = sum_r W_N^{r k} W_R^{r q} (DFT_M x[R m + r])[k]
    template <int K, int Q>
    __device__ static __forceinline__ void comb(cf (&s)[R][M], cf (&x)[N]) {
        if constexpr (K < M) {
            cf t[R];
            twr<K, 0>(s, t);
            dft<R, INV>(t);
#pragma unroll
            for (int q = 0; q < R; ++q) x[K + M * q] = t[q];
            comb<K + 1, 0>(s, x);
        }
    }
    template <int K, int RR>
    __device__ static __forceinline__ void twr(cf (&s)[R][M], cf (&t)[R]) {
        if constexpr (RR < R) {
            t[RR] = rot_n<N, RR * K, INV>(s[RR][K]);
            twr<K, RR + 1>(s, t);
        }
    }
    __device__ static __forceinline__ void run(cf (&x)[N]) {
        if constexpr (N == 2 || N == 3 || N == 4 || N == 5) {
            dft<N, INV>(x);
        } else {
            cf s[R][M];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int m = 0; m < M; ++m) s[r][m] = x[R * m + r];
#pragma unroll
            for (int r = 0; r < R; ++r) RegDft<M, INV>::run(s[r]);
            comb<0, 0>(s, x);
        }
    }
};
template <bool INV>
struct RegDft<1, INV> {
    __device__ static __forceinline__ void run(cf (&)[1]) {}
};

// LDS layout of BATCH sequences of length L.  L % 16 == 0: position p of a
// row lives at p ^ ((p >> 4) & 15) -- an XOR swizzle inside each aligned
// 16-complex block, so the stride-16 Stockham scatters spread over the banks
// while contiguous reads of 32 positions stay one aligned 64-dword block
// (the round-1 pad of one complex per 16 made every such read wrap onto two
// banks: 2x the cycles, tools/lds_banks.py); row pitch RS = L + XRS, XRS
// chosen per kernel for its cross-row (transposing) accesses.  Other L (the
// mixed-radix columns 6..60): pad of one complex per 16.
template <int L, int XRS = 1>
struct Lds {
    // XRS < 0: the padded layout (a kernel whose accesses it suits better)
    static constexpr bool SWZ = (L % 16) == 0 && XRS >= 0;
    // row pitch (complex); the padded pitch is odd so that accesses across
    // rows (one position of many sequences) spread over the banks
    static constexpr int RS = SWZ ? L + XRS : ((L + L / 16 + 1) | 1);
    __device__ static __forceinline__ int at(int b, int p) {
        if constexpr (SWZ) return b * RS + (p ^ ((p >> 4) & 15));
        else return b * RS + p + (p >> 4);
    }
    static constexpr int bytes(int batch) { return batch * RS * 8; }
};

template <int... Rs>
struct RList {};

// LDS byte addressing.  With the swizzled layout, a row pitch RS that is a
// multiple of 16 complex and an LDS buffer aligned to 128 B, the positions a
// Stockham scatter writes -- base + q (Ns = 1) or base + 16 q (Ns = 16) -- sit
// at byte address (A ^ 8q) (+ 128 q): the swizzle XOR of the position's low
// four bits with q folds into ONE v_xor per value on a per-thread byte base
// (the index form costs an XOR and a shift-add per value), and gathers with a
// stride that is a multiple of 256 positions are a base plus immediate
// offsets.  Fft<..., XRS> selects it when Lds<L, XRS>::RS % 16 == 0
// (Fft::XB); the caller then owes the 128-B alignment of the buffer.
typedef float lds_f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) lds_f2 lds_f2_t;
__device__ __forceinline__ uint32_t lds_byte(const cf *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
__device__ __forceinline__ void lds_st(uint32_t a, cf v) {
    lds_f2 w;
    w.x = v.x;
    w.y = v.y;
    *(lds_f2_t *)(uintptr_t)a = w;
}
__device__ __forceinline__ cf lds_ld(uint32_t a) {
    const lds_f2 w = *(const lds_f2_t *)(uintptr_t)a;
    return make_float2(w.x, w.y);
}

// Synchronisation between the Stockham stages' LDS exchanges.  WAVE = true:
// the transform belongs to ONE wave (T = 64 lanes, its own LDS region), so
// the exchange only needs the wave's own LDS operations ordered -- no
// s_barrier: the waves of a workgroup then run their transforms out of step
// with each other, one wave's VALU work covering another's LDS latency.
template <bool WAVE>
__device__ __forceinline__ void stage_sync() {
    if constexpr (WAVE) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
        __syncthreads();
    }
}

// Twiddle table of the radix-16-after-16 stage: tw16[k * kTw16Pitch + q] =
// e^{-2 pi i k q / 256}, k, q < 16 (row pitch 17: rows start on different
// banks).  Filled once per workgroup from kCos256 (correctly rounded fp32,
// below the native sincos' 1.2e-7 error).
static constexpr int kTw16Pitch = 17;
static constexpr int kTw16Size = 16 * kTw16Pitch;
// cos(2 pi m / 256), m = 0..255, correctly rounded to fp32 (float64 cos;
// exactly 0/+-1 at multiples of pi/2)
__device__ constexpr float kCos256[256] = {
    1.000000000e+00f, 9.996988177e-01f, 9.987954497e-01f, 9.972904325e-01f,
    9.951847196e-01f, 9.924795628e-01f, 9.891765118e-01f, 9.852776527e-01f,
    9.807852507e-01f, 9.757021070e-01f, 9.700312614e-01f, 9.637760520e-01f,
    9.569403529e-01f, 9.495281577e-01f, 9.415440559e-01f, 9.329928160e-01f,
    9.238795042e-01f, 9.142097831e-01f, 9.039893150e-01f, 8.932242990e-01f,
    8.819212914e-01f, 8.700869679e-01f, 8.577286005e-01f, 8.448535800e-01f,
    8.314695954e-01f, 8.175848126e-01f, 8.032075167e-01f, 7.883464098e-01f,
    7.730104327e-01f, 7.572088242e-01f, 7.409511209e-01f, 7.242470980e-01f,
    7.071067691e-01f, 6.895405650e-01f, 6.715589762e-01f, 6.531728506e-01f,
    6.343932748e-01f, 6.152315736e-01f, 5.956993103e-01f, 5.758081675e-01f,
    5.555702448e-01f, 5.349976420e-01f, 5.141027570e-01f, 4.928981960e-01f,
    4.713967443e-01f, 4.496113360e-01f, 4.275550842e-01f, 4.052413106e-01f,
    3.826834261e-01f, 3.598950505e-01f, 3.368898630e-01f, 3.136817515e-01f,
    2.902846634e-01f, 2.667127550e-01f, 2.429801822e-01f, 2.191012353e-01f,
    1.950903237e-01f, 1.709618866e-01f, 1.467304677e-01f, 1.224106774e-01f,
    9.801714122e-02f, 7.356456667e-02f, 4.906767607e-02f, 2.454122901e-02f,
    0.000000000e+00f, -2.454122901e-02f, -4.906767607e-02f, -7.356456667e-02f,
    -9.801714122e-02f, -1.224106774e-01f, -1.467304677e-01f, -1.709618866e-01f,
    -1.950903237e-01f, -2.191012353e-01f, -2.429801822e-01f, -2.667127550e-01f,
    -2.902846634e-01f, -3.136817515e-01f, -3.368898630e-01f, -3.598950505e-01f,
    -3.826834261e-01f, -4.052413106e-01f, -4.275550842e-01f, -4.496113360e-01f,
    -4.713967443e-01f, -4.928981960e-01f, -5.141027570e-01f, -5.349976420e-01f,
    -5.555702448e-01f, -5.758081675e-01f, -5.956993103e-01f, -6.152315736e-01f,
    -6.343932748e-01f, -6.531728506e-01f, -6.715589762e-01f, -6.895405650e-01f,
    -7.071067691e-01f, -7.242470980e-01f, -7.409511209e-01f, -7.572088242e-01f,
    -7.730104327e-01f, -7.883464098e-01f, -8.032075167e-01f, -8.175848126e-01f,
    -8.314695954e-01f, -8.448535800e-01f, -8.577286005e-01f, -8.700869679e-01f,
    -8.819212914e-01f, -8.932242990e-01f, -9.039893150e-01f, -9.142097831e-01f,
    -9.238795042e-01f, -9.329928160e-01f, -9.415440559e-01f, -9.495281577e-01f,
    -9.569403529e-01f, -9.637760520e-01f, -9.700312614e-01f, -9.757021070e-01f,
    -9.807852507e-01f, -9.852776527e-01f, -9.891765118e-01f, -9.924795628e-01f,
    -9.951847196e-01f, -9.972904325e-01f, -9.987954497e-01f, -9.996988177e-01f,
    -1.000000000e+00f, -9.996988177e-01f, -9.987954497e-01f, -9.972904325e-01f,
    -9.951847196e-01f, -9.924795628e-01f, -9.891765118e-01f, -9.852776527e-01f,
    -9.807852507e-01f, -9.757021070e-01f, -9.700312614e-01f, -9.637760520e-01f,
    -9.569403529e-01f, -9.495281577e-01f, -9.415440559e-01f, -9.329928160e-01f,
    -9.238795042e-01f, -9.142097831e-01f, -9.039893150e-01f, -8.932242990e-01f,
    -8.819212914e-01f, -8.700869679e-01f, -8.577286005e-01f, -8.448535800e-01f,
    -8.314695954e-01f, -8.175848126e-01f, -8.032075167e-01f, -7.883464098e-01f,
    -7.730104327e-01f, -7.572088242e-01f, -7.409511209e-01f, -7.242470980e-01f,
    -7.071067691e-01f, -6.895405650e-01f, -6.715589762e-01f, -6.531728506e-01f,
    -6.343932748e-01f, -6.152315736e-01f, -5.956993103e-01f, -5.758081675e-01f,
    -5.555702448e-01f, -5.349976420e-01f, -5.141027570e-01f, -4.928981960e-01f,
    -4.713967443e-01f, -4.496113360e-01f, -4.275550842e-01f, -4.052413106e-01f,
    -3.826834261e-01f, -3.598950505e-01f, -3.368898630e-01f, -3.136817515e-01f,
    -2.902846634e-01f, -2.667127550e-01f, -2.429801822e-01f, -2.191012353e-01f,
    -1.950903237e-01f, -1.709618866e-01f, -1.467304677e-01f, -1.224106774e-01f,
    -9.801714122e-02f, -7.356456667e-02f, -4.906767607e-02f, -2.454122901e-02f,
    0.000000000e+00f, 2.454122901e-02f, 4.906767607e-02f, 7.356456667e-02f,
    9.801714122e-02f, 1.224106774e-01f, 1.467304677e-01f, 1.709618866e-01f,
    1.950903237e-01f, 2.191012353e-01f, 2.429801822e-01f, 2.667127550e-01f,
    2.902846634e-01f, 3.136817515e-01f, 3.368898630e-01f, 3.598950505e-01f,
    3.826834261e-01f, 4.052413106e-01f, 4.275550842e-01f, 4.496113360e-01f,
    4.713967443e-01f, 4.928981960e-01f, 5.141027570e-01f, 5.349976420e-01f,
    5.555702448e-01f, 5.758081675e-01f, 5.956993103e-01f, 6.152315736e-01f,
    6.343932748e-01f, 6.531728506e-01f, 6.715589762e-01f, 6.895405650e-01f,
    7.071067691e-01f, 7.242470980e-01f, 7.409511209e-01f, 7.572088242e-01f,
    7.730104327e-01f, 7.883464098e-01f, 8.032075167e-01f, 8.175848126e-01f,
    8.314695954e-01f, 8.448535800e-01f, 8.577286005e-01f, 8.700869679e-01f,
    8.819212914e-01f, 8.932242990e-01f, 9.039893150e-01f, 9.142097831e-01f,
    9.238795042e-01f, 9.329928160e-01f, 9.415440559e-01f, 9.495281577e-01f,
    9.569403529e-01f, 9.637760520e-01f, 9.700312614e-01f, 9.757021070e-01f,
    9.807852507e-01f, 9.852776527e-01f, 9.891765118e-01f, 9.924795628e-01f,
    9.951847196e-01f, 9.972904325e-01f, 9.987954497e-01f, 9.996988177e-01f};
__device__ __forceinline__ void tw16_fill(cf *tw16, int tid, int nthreads) {
    for (int i = tid; i < 256; i += nthreads) {
        const int k = i >> 4, q = i & 15, m = k * q;             // m < 256
        tw16[k * kTw16Pitch + q] = make_float2(kCos256[m], -kCos256[(m + 192) & 255]);
    }
}

template <int L, int BATCH, int T, bool WAVE = false, int XRS = 1>
struct Fft {
    using LD = Lds<L, XRS>;
    // byte-address forms of the exchanges (see lds_byte)
    static constexpr bool XB = LD::SWZ && (LD::RS % 16 == 0);
    static constexpr int E = L * BATCH / T;
    static_assert(E * T == L * BATCH, "T must divide L*BATCH");
    static_assert(!WAVE || (T == 64 && BATCH == 1), "a wave-local transform is one sequence on 64 lanes");

    // Fill registers with the first-stage INPUT mapping of radix R0 from LDS.
    template <int R0>
    __device__ static __forceinline__ void load(cf (&v)[E], const cf *lds, int tid) {
        constexpr int LR = L / R0;
#pragma unroll
        for (int ib = 0; ib < E / R0; ++ib) {
            const int j = tid + ib * T, b = j / LR, jj = j - b * LR;
            if constexpr (XB && LR % 256 == 0) {
                // positions jj + q LR: the swizzle XOR (jj >> 4) & 15 is the same for every q
                const uint32_t a = lds_byte(lds) + 8u * (uint32_t)LD::at(b, jj);
#pragma unroll
                for (int q = 0; q < R0; ++q) v[ib * R0 + q] = lds_ld(a + 8u * (uint32_t)(q * LR));
            } else {
#pragma unroll
                for (int q = 0; q < R0; ++q) v[ib * R0 + q] = lds[LD::at(b, jj + q * LR)];
            }
        }
    }
    // Store registers (last-stage OUTPUT mapping of radix R) to LDS, natural.
    template <int R>
    __device__ static __forceinline__ void store(const cf (&v)[E], cf *lds, int tid) {
        constexpr int LR = L / R;
#pragma unroll
        for (int ib = 0; ib < E / R; ++ib) {
            const int j = tid + ib * T, b = j / LR, jj = j - b * LR;
#pragma unroll
            for (int q = 0; q < R; ++q) lds[LD::at(b, jj + q * LR)] = v[ib * R + q];
        }
    }
    // (b, position) of register i under the natural mapping of radix R.
    template <int R>
    __device__ static __forceinline__ void where(int i, int tid, int &b, int &pos) {
        constexpr int LR = L / R;
        const int ib = i / R, q = i - ib * R;
        const int j = tid + ib * T;
        b = j / LR;
        pos = j - b * LR + q * LR;
    }

    // Run the stage list.  Ns = product of the radices already applied.
    template <bool INV, int Ns, int R, int... Rest>
    __device__ static __forceinline__ void run(cf (&v)[E], cf *lds, int tid) {
        run_impl<INV, false, false, Ns, R, Rest...>(v, lds, tid, nullptr);
    }
    // The same with the radix-16 stage after a radix-16 stage (Ns = 16: the
    // 15 twiddles w^q, w = e^{-+2 pi i k/256}, k < 16) read from the table
    // tw16[k * kTw16Pitch + q] = e^{-2 pi i k q / 256} (tw16_fill) instead of
    // 4 native sincos + 11 products per butterfly.
    template <bool INV, int Ns, int R, int... Rest>
    __device__ static __forceinline__ void run_tw(cf (&v)[E], cf *lds, int tid, const cf *tw16) {
        run_impl<INV, true, false, Ns, R, Rest...>(v, lds, tid, tw16);
    }

    // Every stage but the last, then the exchange into the last stage's input
    // mapping: the caller runs the last stage itself (pass A merges the
    // four-step twiddle into it).  Ns of the last stage = L / (its radix).
    template <bool INV, int Ns, int R, int... Rest>
    __device__ static __forceinline__ void run_head_tw(cf (&v)[E], cf *lds, int tid, const cf *tw16) {
        static_assert(sizeof...(Rest) >= 1, "run_head_tw needs at least two stages");
        run_impl<INV, true, true, Ns, R, Rest...>(v, lds, tid, tw16);
    }

    template <bool INV, bool TW, bool HEAD, int Ns, int R, int... Rest>
    __device__ static __forceinline__ void run_impl(cf (&v)[E], cf *lds, int tid, const cf *tw16) {
        static_assert(E % R == 0, "E must be a multiple of every radix");
        constexpr int LR = L / R;
#pragma unroll
        for (int ib = 0; ib < E / R; ++ib) {
            const int j = tid + ib * T, b = j / LR, jj = j - b * LR;
            const int k = jj % Ns;
            cf *a = v + ib * R;
            if constexpr (TW && Ns == 16 && R == 16) {
                const cf *t = tw16 + k * kTw16Pitch;
#pragma unroll
                for (int q = 1; q < 16; ++q) a[q] = INV ? cmul_conj(a[q], t[q]) : cmul(a[q], t[q]);
            } else if constexpr (Ns > 1) {
                // a[q] *= w^q, w = exp(-+2 pi i k / (Ns R)).  w^(2^j) from the
                // native trig (angles < 1/2 rev), the other powers as products
                // of at most four of those (<= 3 roundings).
                constexpr int H = (R >= 8) ? R / 2 : R;   // powers kept: w^1 .. w^(H-1)
                cf w[H];
                const float base = (float)k * (1.0f / (float)(Ns * R));   // [0, 1/R)
#pragma unroll
                for (int p2 = 1; p2 < H; p2 *= 2) w[p2] = expi_rev(INV ? p2 * base : -p2 * base);
#pragma unroll
                for (int q = 3; q < H; ++q) {
                    const int hi = 1 << (31 - __builtin_clz(q));   // compile-time after unrolling
                    if (q != hi) w[q] = cmul(w[hi], w[q - hi]);
                }
#pragma unroll
                for (int q = 1; q < H; ++q) a[q] = cmul(a[q], w[q]);
                if constexpr (H < R) {
                    const cf wh = expi_rev(INV ? H * base : -H * base);
                    a[H] = cmul(a[H], wh);
#pragma unroll
                    for (int q = 1; q < H; ++q) a[H + q] = cmul(a[H + q], cmul(wh, w[q]));
                }
            }
            dft<R, INV>(a);
        }
        if constexpr (sizeof...(Rest) > 0) {
            // Stockham scatter of this stage's outputs, then gather the next
            // stage's inputs.
#pragma unroll
            for (int ib = 0; ib < E / R; ++ib) {
                const int j = tid + ib * T, b = j / LR, jj = j - b * LR;
                const int k = jj % Ns;
                const int base = (jj / Ns) * Ns * R + k;
                if constexpr (XB && 16 % R == 0 && Ns == 1) {
                    // positions base + q, base = R jj: at = X ^ q
                    const uint32_t a = lds_byte(lds) + 8u * (uint32_t)(b * LD::RS + (base ^ ((base >> 4) & 15)));
#pragma unroll
                    for (int q = 0; q < R; ++q) lds_st(a ^ (8u * (uint32_t)q), v[ib * R + q]);
                } else if constexpr (XB && 16 % R == 0 && Ns == 16) {
                    // positions base + 16 q, base = 16 R G + k (G = jj / 16):
                    // the swizzle XOR is c | q, c = (R G) & 15, so at = (X ^ q) + 16 q
                    // with X = b RS + (base ^ c)
                    const int c = ((jj / Ns) * R) & 15;
                    const uint32_t a = lds_byte(lds) + 8u * (uint32_t)(b * LD::RS + (base ^ c));
#pragma unroll
                    for (int q = 0; q < R; ++q) lds_st((a ^ (8u * (uint32_t)q)) + 128u * (uint32_t)q, v[ib * R + q]);
                } else if constexpr (XB && Ns % 256 == 0) {
                    // positions base + Ns q: the swizzle XOR is the same for every q
                    const uint32_t a = lds_byte(lds) + 8u * (uint32_t)LD::at(b, base);
#pragma unroll
                    for (int q = 0; q < R; ++q) lds_st(a + 8u * (uint32_t)(q * Ns), v[ib * R + q]);
                } else {
#pragma unroll
                    for (int q = 0; q < R; ++q) lds[LD::at(b, base + q * Ns)] = v[ib * R + q];
                }
            }
            stage_sync<WAVE>();
            constexpr int R2 = first<Rest...>();
            load<R2>(v, lds, tid);
            stage_sync<WAVE>();
            if constexpr (!(HEAD && sizeof...(Rest) == 1)) run_impl<INV, TW, HEAD, Ns * R, Rest...>(v, lds, tid, tw16);
        }
    }

    template <int A, int... Z>
    static constexpr int first() { return A; }
    template <int... Z>
    static constexpr int last_of() {
        constexpr int a[] = {Z...};
        return a[sizeof...(Z) - 1];
    }
};

}  // namespace pss
