// host_asan.cpp -- AddressSanitizer / UBSan driver for the native host
// planning code (psrsigsim_amd/csrc/pss_host.cpp, SURVEY.md §5 "Race detection
// / sanitizers": build-time -fsanitize=address host tests).
//
// Built with g++ -fsanitize=address,undefined together with pss_host.cpp by
// tests/test_host_asan.py and run as a child process.  Exercises every entry
// point at edge sizes (K = 2, 3; rows 0, 1, below and above the threading
// threshold; n = 0; phases outside the knot range; NaN/flat data) on exactly
// sized heap buffers, so any out-of-bounds access trips ASan, and checks the
// results against straightforward reimplementations (PCHIP interpolates its
// knots; the device table is c * (h^3, h^2, h, 1) / amax).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/pss_hip.h"

static int g_fail = 0;
#define CHECK(c, ...)                                              \
    do {                                                           \
        if (!(c)) {                                                \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);   \
            fprintf(stderr, __VA_ARGS__);                          \
            fprintf(stderr, "\n");                                 \
            ++g_fail;                                              \
        }                                                          \
    } while (0)

static double urand(unsigned &s) {
    s = s * 1664525u + 1013904223u;
    return (double)(s >> 8) / (double)(1u << 24);
}

// exactly sized heap copies: ASan sees one-past-the-end accesses
template <typename T>
static T *dup(const std::vector<T> &v) {
    T *p = (T *)malloc(v.size() * sizeof(T) + (v.empty() ? 1 : 0));
    if (!v.empty()) memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

static void case_pchip(int64_t K, int64_t rows, int nthreads, int kind) {
    unsigned s = (unsigned)(K * 131 + rows * 7 + kind);
    std::vector<double> x(K), y(K * rows);
    for (int64_t i = 0; i < K; ++i) x[i] = (double)i / (double)(K - 1);
    for (int64_t r = 0; r < rows; ++r)
        for (int64_t i = 0; i < K; ++i) {
            double v = urand(s);
            if (kind == 1) v = 0.5;                         // flat rows
            if (kind == 2 && i % 3 == 0) v = 0.0;           // zero slopes
            if (kind == 3 && i == K / 2) v = NAN;           // a NaN knot
            y[r * K + i] = v;
        }
    double *xp = dup(x), *yp = dup(y);
    double *c = (double *)malloc(sizeof(double) * (rows * (K - 1) * 4 + 1));
    CHECK(pss_host_pchip_coef(xp, K, yp, rows, c, nthreads) == PSS_OK, "pchip_coef K=%lld rows=%lld",
          (long long)K, (long long)rows);
    // evaluate at the knots (and beyond both ends: extrapolation)
    const int64_t n = K + 2;
    std::vector<double> ph(n);
    ph[0] = -0.25;
    for (int64_t i = 0; i < K; ++i) ph[i + 1] = x[i];
    ph[K + 1] = 1.5;
    double *php = dup(ph);
    double *out = (double *)malloc(sizeof(double) * (rows * n + 1));
    CHECK(pss_host_ppoly_eval(xp, K, c, rows, php, n, out, nthreads) == PSS_OK, "ppoly_eval");
    for (int64_t r = 0; r < rows; ++r)
        for (int64_t i = 0; i + 1 < K; ++i) {            // the last knot is reached by the last piece
            const double want = y[r * K + i], got = out[r * n + i + 1];
            if (kind == 3) continue;
            CHECK(fabs(got - want) <= 1e-12, "knot r=%lld i=%lld got %.17g want %.17g", (long long)r,
                  (long long)i, got, want);
        }
    // device table
    const double h = 1.0 / (double)(K - 1), amax = kind == 1 ? 1.0 : 0.75;
    float *tab = (float *)malloc(sizeof(float) * (rows * (K - 1) * 4 + 1));
    CHECK(pss_host_device_table(c, rows, K - 1, h, amax, tab, nthreads) == PSS_OK, "device_table");
    const double w[4] = {h * h * h, h * h, h, 1.0};
    for (int64_t e = 0; e < rows * (K - 1) * 4; ++e) {
        const float want = (float)(c[e] * w[e & 3] / amax);
        if (kind == 3) continue;
        CHECK(fabsf(tab[e] - want) <= 1e-6f * (fabsf(want) + 1e-30f), "table e=%lld", (long long)e);
    }
    free(xp);
    free(yp);
    free(c);
    free(php);
    free(out);
    free(tab);
}

int main() {
    const int64_t Ks[] = {2, 3, 4, 5, 17, 245, 1025};
    const int64_t Rs[] = {0, 1, 2, 63, 64, 65, 200};
    for (int64_t K : Ks)
        for (int64_t R : Rs)
            for (int th : {1, 4})
                for (int kind = 0; kind < 4; ++kind) case_pchip(K, R, th, kind);
    // argument validation
    double d = 0.0;
    float f = 0.f;
    CHECK(pss_host_pchip_coef(&d, 1, &d, 1, &d, 1) == PSS_EINVAL, "K < 2 accepted");
    CHECK(pss_host_pchip_coef(nullptr, 3, &d, 1, &d, 1) == PSS_EINVAL, "NULL x accepted");
    CHECK(pss_host_ppoly_eval(&d, 1, &d, 1, &d, 1, &d, 1) == PSS_EINVAL, "ppoly K < 2 accepted");
    CHECK(pss_host_ppoly_eval(&d, 2, &d, 1, &d, -1, &d, 1) == PSS_EINVAL, "ppoly n < 0 accepted");
    CHECK(pss_host_device_table(&d, 1, 0, 1.0, 1.0, &f, 1) == PSS_EINVAL, "nint < 1 accepted");
    // n = 0 phases: nothing written, no access
    CHECK(pss_host_ppoly_eval(&d, 2, &d, 1, &d, 0, &d, 1) == PSS_OK, "ppoly n = 0");
    if (g_fail) {
        fprintf(stderr, "%d failures\n", g_fail);
        return 1;
    }
    printf("host_asan: ok\n");
    return 0;
}
