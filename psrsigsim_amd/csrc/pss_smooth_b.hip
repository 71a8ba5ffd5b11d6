// pss_smooth_b.hip -- mixed-radix four-step, N1 = 24, 30 (fold-mode C4's 30 x 1024), 40.
#include "pss_engine.hpp"

using namespace pss;

int run_smooth_b(KP &k, hipStream_t st) {
    switch (k.N1) {
        case 24: return launch_smooth_n2<24, RList<2, 4, 3>, RList<3, 4, 2>, 256>(k, st);
        case 30: return launch_smooth_n2<30, RList<2, 3, 5>, RList<5, 3, 2>, 256>(k, st);
        case 40: return launch_smooth_n2<40, RList<2, 4, 5>, RList<5, 4, 2>, 128>(k, st);
        default: return fail(PSS_EUNSUPPORTED, "N1=%lld", (long long)k.N1);
    }
}
