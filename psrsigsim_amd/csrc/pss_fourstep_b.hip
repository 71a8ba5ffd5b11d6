// pss_fourstep_b.hip -- the power-of-two four-step lengths other than C3's 2^22
// (2^14 .. 2^21, 2^23, 2^24), compiled in parallel with pss_fourstep.hip.
#include "pss_engine.hpp"

using namespace pss;

int run_fourstep_b(KP &k, hipStream_t st, const float *mask_row) {
    const int64_t N = k.N;
    if (N == (1 << 23)) {
        k.N2 = 8192;
        k.N1 = 1024;
        return launch_pair<1024, 8, 512, C1kF, C1kF, 8192, 1024, C8kF, C8kI, 512>(k, st, mask_row);
    }
    if (N == (1 << 24)) {
        if (k.p.null_mode != PSS_NULL_DELAYED && !k.p.htab && !k.p.tail_a) {
            // C5: 1024 x 16384 -- C3's column kernels (1024-point columns:
            // pass A two workgroups per CU, pass C 16-column blocks) and a
            // one-row-at-a-time 16384-point row pass (PairRowsSeq, 1024
            // threads, 133 KB of LDS)
            k.N2 = 16384;
            k.N1 = 1024;
            return launch_pair<1024, 8, 512, C1kF, C1kF, 16384, 1024, C16kF, C16kI, 1024, kBC, kTC>(k, st, mask_row);
        }
        // with a delayed null (the mask table's row engine holds a pair of
        // rows), a transfer function or the tail: 2048 x 8192.  Pass A: the
        // LDS-staged fast kernel on 2048-point columns; pass C: 16-column
        // register-resident blocks (passC_fast32)
        k.N2 = 8192;
        k.N1 = 2048;
        return launch_pair<2048, 8, 512, C2kF, C2kF, 8192, 1024, C8kF, C8kI, 512, 8, 1024>(k, st, mask_row);
    }
    if (N >= (1 << 17)) {
        // 2^17 .. 2^21: rows of 4096 (the C3 row kernel: two rows of a pair
        // in 66 KB, two workgroups per CU) and N / 4096 columns; the column
        // kernels keep their 8192 / N1-column blocks (N2 / B >= 16 per pair)
        k.N2 = 4096;
        k.N1 = N / 4096;
        switch (k.N1) {
#define CASE4K(N1_, CF, CI)                                                                          \
    case N1_:                                                                                        \
        return launch_pair<N1_, 8192 / N1_, 512, CF, CF, 4096, 512, C4k, C4k, 256>(k, st, mask_row);
            CASE4K(32, C32F, C32I)
            CASE4K(64, C64F, C64I)
            CASE4K(128, C128F, C128I)
            CASE4K(256, C256, C256)
            CASE4K(512, C512F, C512I)
#undef CASE4K
            default: break;
        }
        return fail(PSS_EUNSUPPORTED, "four-step: N=%lld", (long long)N);
    }
    // 2^14 .. 2^16: N1 = 16 columns, rows of N/16
    k.N1 = 16;
    k.N2 = N / 16;
    switch (k.N2) {
        case 1024:
            return launch_pair<16, 512, 512, C16, C16, 1024, 128, C1kF, C1kI, 64>(k, st, mask_row);
        case 2048:
            return launch_pair<16, 512, 512, C16, C16, 2048, 256, C2kF, C2kI, 128>(k, st, mask_row);
        case 4096:
            return launch_pair<16, 512, 512, C16, C16, 4096, 512, C4k, C4k, 256>(k, st, mask_row);
        default: break;
    }
    return fail(PSS_EUNSUPPORTED, "four-step: N=%lld", (long long)N);
}

