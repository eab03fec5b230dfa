// Dumps make_plan's k_pyramid tiling (orbx_geometry.h) for one configuration:
//   pyramid_plan W H nfeatures nlevels
// prints "L nseg", per segment "l0 nl nx ny lds_a lds_b", one line per level "w h" plus
// its resize tables, then per segment, tile and segment level "x0 y0 x1 y1 ox0 oy0 ox1 oy1".  tests/test_pyramid_plan.py checks
// the invariants k_pyramid relies on.
#include <cstdio>
#include <cstdlib>

#include "orbx_geometry.h"

using namespace orbx;

int main(int argc, char** argv) {
    if (argc < 5) return 2;
    const int W = std::atoi(argv[1]), H = std::atoi(argv[2]), nf = std::atoi(argv[3]), L = std::atoi(argv[4]);
    OrbParams p;
    if (!init_params(p, nf, 1.2f, L, 20, 7)) return 3;
    Plan pl;
    if (!make_plan(pl, p, W, H)) {
        std::printf("FAIL %s\n", pl.why ? pl.why : "");
        return 4;
    }
    std::printf("%d %d\n", pl.L, pl.pz_nseg);
    for (int s = 0; s < pl.pz_nseg; s++)
        std::printf("%d %d %d %d %d %d\n", pl.pz[s].l0, pl.pz[s].nl, pl.pz[s].nx, pl.pz[s].ny, pl.pz[s].lds_a,
                    pl.pz[s].lds_b);
    for (int l = 0; l < pl.L; l++) {
        const LevelGeom& g = pl.lv[l];
        std::printf("%d %d\n", g.w, g.h);
        if (l > 0) {
            const int16_t* xt = pl.rtab.data() + g.xtab_off;
            const int16_t* yt = pl.rtab.data() + g.ytab_off;
            for (int x = 0; x < g.w; x++) std::printf("%d %d ", xt[4 * x], xt[4 * x + 1]);
            std::printf("\n");
            for (int y = 0; y < g.h; y++) std::printf("%d %d ", yt[4 * y], yt[4 * y + 1]);
            std::printf("\n");
        }
    }
    for (int s = 0; s < pl.pz_nseg; s++)
        for (int t = 0; t < pl.pz[s].tiles; t++)
            for (int k = 0; k < pl.pz[s].nl; k++) {
                const int16_t* R = pl.rtab.data() + pl.pz[s].off + ((size_t)t * pl.pz[s].nl + k) * 8;
                std::printf("%d %d %d %d %d %d %d %d\n", R[0], R[1], R[2], R[3], R[4], R[5], R[6], R[7]);
            }
    return 0;
}
