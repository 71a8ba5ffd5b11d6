// pss_smooth.hip -- the mixed-radix four-step (2^m x {6..60}, 1250 x 2500):
// the dispatch and N1 = 6 .. 20 (the other column lengths: pss_smooth_b/c.hip,
// compiled in parallel).
#include "pss_engine.hpp"

using namespace pss;

int run_smooth(KP &k, hipStream_t st) {
    int64_t n1 = 0, n2 = 0;
    if (!smooth_split(k.N, &n1, &n2)) return fail(PSS_EUNSUPPORTED, "N=%lld", (long long)k.N);
    k.N1 = n1;
    k.N2 = n2;
    plan_note("smooth");
    switch (n1) {
        case 6:  return launch_smooth_n2<6, RList<2, 3>, RList<3, 2>, 256>(k, st);
        case 10: return launch_smooth_n2<10, RList<2, 5>, RList<5, 2>, 256>(k, st);
        case 12: return launch_smooth_n2<12, RList<4, 3>, RList<3, 4>, 256>(k, st);
        case 20: return launch_smooth_n2<20, RList<4, 5>, RList<5, 4>, 256>(k, st);
        case 24: case 30: case 40: return run_smooth_b(k, st);
        default: return run_smooth_c(k, st);
    }
}
