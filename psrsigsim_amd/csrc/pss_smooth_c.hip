// pss_smooth_c.hip -- mixed-radix four-step, N1 = 48, 60 and 3 125 000 = 1250 x 2500.
#include "pss_engine.hpp"

using namespace pss;

int run_smooth_c(KP &k, hipStream_t st) {
    if (k.N1 == 1250 && k.N2 == 2500) {
        // 4-column blocks (2500 = 4 x 625) of 250 threads, 20 values each
        using C1250 = RList<2, 5, 5, 5, 5>;
        return launch_pair<1250, 4, 250, C1250, C1250, 2500, 250, RList<5, 5, 5, 5, 4>, RList<4, 5, 5, 5, 5>, 250, 4,
                           250>(k, st, nullptr);
    }
    switch (k.N1) {
        case 48: return launch_smooth_n2<48, RList<4, 4, 3>, RList<3, 4, 4>, 128>(k, st);
        case 60: return launch_smooth_n2<60, RList<4, 3, 5>, RList<5, 3, 4>, 128>(k, st);
        default: return fail(PSS_EUNSUPPORTED, "N1=%lld", (long long)k.N1);
    }
}
