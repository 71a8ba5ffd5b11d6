// pss_single.hip -- N = 2^m <= 8192: a row (or rows) per workgroup in LDS.
#include "pss_engine.hpp"

using namespace pss;

static int launch_single_n(KP &k, hipStream_t st) {
    switch (k.N) {
        case 64: return launch_single<64, 64, 256, C64F, C64I>(k, st);
        case 128: return launch_single<128, 32, 256, C128F, C128I>(k, st);
        case 256: return launch_single<256, 16, 256, C256, C256>(k, st);
        case 512: return launch_single<512, 8, 256, C512F, C512I>(k, st);
        case 1024: return launch_single<1024, 4, 256, C1kF, C1kI>(k, st);
        case 2048: return launch_single<2048, 2, 256, C2kF, C2kI>(k, st);
        case 4096: return launch_single<4096, 1, 256, C4k, C4k>(k, st);
        case 8192: return launch_single<8192, 1, 512, C8kF, C8kI>(k, st);
        default: break;
    }
    return fail(PSS_EUNSUPPORTED, "single-pass: N=%lld", (long long)k.N);
}

int run_single(KP &k, hipStream_t st) {
    k.N1 = 1;
    k.N2 = k.N;
    if (!refine_null(k)) return launch_single_n(k, st);
    // a delayed null decided in float64: the kernel leaves
    // (data, mask) per sample in W1, the samples within the fp32 error of the
    // threshold are re-decided from the box row's float64 spectrum
    // (launch_null_refine), then the epilogue (null, observe copy, noise, store)
    k.w1_out = reinterpret_cast<cf *>(k.p.work);
    int rc = launch_single_n(k, st);
    if (!rc) rc = launch_null_refine(k, st);
    if (!rc) rc = launch_fb_epilogue(k, st);
    return rc;
}

