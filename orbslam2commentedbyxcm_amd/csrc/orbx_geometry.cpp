// orbx_geometry.cpp -- host-side extraction plan (see orbx_geometry.h).
// Compiled with -ffp-contract=off: every float expression below restates a
// reference expression operation by operation.
#include <algorithm>
#include "orbx_geometry.h"
#include "orbx_error.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace orbx {

static int cv_round(double v) { return (int)std::lrint(v); }   // cvRound: round half to even
static int cv_roundf(float v) { return (int)std::lrintf(v); }

// ORBextractor::ORBextractor, ORBextractor.cc:438-550
bool init_params(OrbParams& p, int nfeatures, float scale_factor, int nlevels, int ini, int min) {
    if (nlevels < 1 || nlevels > kMaxLevels || nfeatures < 0 || !(scale_factor > 1.0f)) return false;
    p.nfeatures = nfeatures;
    p.scale_factor = (double)scale_factor;
    p.nlevels = nlevels;
    p.ini_th = ini;
    p.min_th = min;
    p.scale[0] = 1.0f;
    p.sigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
        p.scale[i] = (float)((double)p.scale[i - 1] * p.scale_factor);   // cc:458
        p.sigma2[i] = p.scale[i] * p.scale[i];                            // cc:460
    }
    for (int i = 0; i < nlevels; i++) {
        p.inv_scale[i] = 1.0f / p.scale[i];                               // cc:468
        p.inv_sigma2[i] = 1.0f / p.sigma2[i];                             // cc:469
    }
    const float factor = (float)(1.0f / p.scale_factor);                   // cc:480
    float desired = (float)nfeatures * (1 - factor) /
                    (1 - (float)std::pow((double)factor, (double)nlevels));  // cc:485
    int sum = 0;
    for (int level = 0; level < nlevels - 1; level++) {                    // cc:490-498
        p.features[level] = cv_roundf(desired);
        sum += p.features[level];
        desired *= factor;
    }
    p.features[nlevels - 1] = nfeatures - sum > 0 ? nfeatures - sum : 0;  // cc:500
    // umax, cc:519-549
    const int vmax = (int)std::floor(15 * std::sqrt(2.f) / 2 + 1);
    const int vmin = (int)std::ceil(15 * std::sqrt(2.f) / 2);
    const double hp2 = 15 * 15;
    int v, v0;
    for (v = 0; v <= vmax; ++v) p.umax[v] = cv_round(std::sqrt(hp2 - v * v));
    for (v = 15, v0 = 0; v >= vmin; --v) {
        while (p.umax[v0] == p.umax[v0 + 1]) ++v0;
        p.umax[v] = v0;
        ++v0;
    }
    return true;
}

// OpenCV 3.3.1 resize(INTER_LINEAR) coefficient tables for CV_8U (11-bit fixed point).
static void resize_tables(int sw, int sh, int dw, int dh, int16_t* xtab, int16_t* ytab) {
    const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    int xmax = dw;
    std::vector<int> sxs(dw);
    std::vector<float> fxs(dw);
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        sxs[dx] = sx;
        fxs[dx] = fx;
    }
    for (int dx = 0; dx < dw; dx++) {
        int16_t* t = xtab + 4 * dx;
        if (dx < xmax) {
            t[0] = (int16_t)sxs[dx];
            t[1] = (int16_t)(sxs[dx] + 1);
            t[2] = (int16_t)cv_roundf((1.f - fxs[dx]) * 2048);
            t[3] = (int16_t)cv_roundf(fxs[dx] * 2048);
        } else {  // HResizeLinear tail: D = S[sx] * INTER_RESIZE_COEF_SCALE
            t[0] = (int16_t)sxs[dx];
            t[1] = (int16_t)sxs[dx];
            t[2] = 2048;
            t[3] = 0;
        }
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)std::floor(fy);
        fy -= sy;
        int16_t* t = ytab + 4 * dy;
        auto clip = [&](int y) { return y < 0 ? 0 : (y >= sh ? sh - 1 : y); };
        t[0] = (int16_t)clip(sy);
        t[1] = (int16_t)clip(sy + 1);
        t[2] = (int16_t)cv_roundf((1.f - fy) * 2048);
        t[3] = (int16_t)cv_roundf(fy * 2048);
    }
}

// k_pyramid tile rectangles (orbx_geometry.h).  Ownership: level 0 is split into an
// nx x ny grid; a boundary b at level l - 1 moves to the first level-l column (row)
// whose resize source starts at or after b, so a tile's owned pixels at level l read
// only its own pixels at level l - 1 apart from the one-pixel right / bottom reach of
// the interpolation.  Needed rectangles are then grown from the top level down by the
// resize tables' source footprints (the tables are monotone, so a range of columns
// maps to [t(first).s0, t(last).s1]): the halo is 0 on the left / top and about
// 1 + 1.2 * (halo of the level above) on the right / bottom.
// One segment: levels s.l0 .. s.l0 + s.nl - 1, tiled over level s.l0 (owned by the
// segment only when s.l0 == 0: a later segment's input level is already in HBM).
static bool pyramid_segment(Plan& plan, PzSeg& s, int tw, int th) {
    const int l0 = s.l0, n = s.nl;
    const LevelGeom& g0 = plan.lv[l0];
    const int nx = (g0.w + tw - 1) / tw, ny = (g0.h + th - 1) / th;
    s.nx = nx;
    s.ny = ny;
    s.tiles = nx * ny;
    s.off = (int)plan.rtab.size();
    plan.rtab.resize(plan.rtab.size() + (size_t)nx * ny * n * 8);
    // owned boundaries per segment level: bx[k][0..nx], by[k][0..ny] (level l0 + k)
    std::vector<std::vector<int>> bx(n, std::vector<int>(nx + 1)), by(n, std::vector<int>(ny + 1));
    for (int j = 0; j <= nx; j++) bx[0][j] = (int)(((long long)j * g0.w) / nx);
    for (int i = 0; i <= ny; i++) by[0][i] = (int)(((long long)i * g0.h) / ny);
    for (int k = 1; k < n; k++) {
        const LevelGeom& g = plan.lv[l0 + k];
        const int16_t* xt = plan.rtab.data() + g.xtab_off;
        const int16_t* yt = plan.rtab.data() + g.ytab_off;
        for (int j = 0; j <= nx; j++) {
            int c = j == 0 ? 0 : bx[k][j - 1];
            while (c < g.w && (j == nx || xt[4 * c] < bx[k - 1][j])) c++;
            bx[k][j] = c;
        }
        for (int i = 0; i <= ny; i++) {
            int r = i == 0 ? 0 : by[k][i - 1];
            while (r < g.h && (i == ny || yt[4 * r] < by[k - 1][i])) r++;
            by[k][i] = r;
        }
    }
    for (int ty = 0; ty < ny; ty++)
        for (int tx = 0; tx < nx; tx++) {
            int16_t* R = plan.rtab.data() + s.off + (size_t)(ty * nx + tx) * n * 8;
            int nx0 = 0, ny0 = 0, nx1 = 0, ny1 = 0;  // needed rectangle of level l + 1
            for (int k = n - 1; k >= 0; k--) {
                const int l = l0 + k;
                int ox0 = bx[k][tx], ox1 = bx[k][tx + 1], oy0 = by[k][ty], oy1 = by[k][ty + 1];
                if (k == 0 && l0 > 0) ox0 = ox1 = oy0 = oy1 = 0;  // the input level: not owned here
                int x0 = ox0, x1 = ox1, y0 = oy0, y1 = oy1;
                bool any = ox1 > ox0 && oy1 > oy0;
                if (k + 1 < n && nx1 > nx0 && ny1 > ny0) {
                    const LevelGeom& u = plan.lv[l + 1];
                    const int16_t* xt = plan.rtab.data() + u.xtab_off;
                    const int16_t* yt = plan.rtab.data() + u.ytab_off;
                    const int sx0 = xt[4 * nx0], sx1 = xt[4 * (nx1 - 1) + 1] + 1;
                    const int sy0 = yt[4 * ny0], sy1 = yt[4 * (ny1 - 1) + 1] + 1;
                    if (any) {
                        x0 = std::min(x0, sx0); x1 = std::max(x1, sx1);
                        y0 = std::min(y0, sy0); y1 = std::max(y1, sy1);
                    } else {
                        x0 = sx0; x1 = sx1; y0 = sy0; y1 = sy1;
                    }
                    any = true;
                }
                if (!any) x0 = x1 = y0 = y1 = 0;
                const int16_t r[8] = {(int16_t)x0, (int16_t)y0, (int16_t)x1, (int16_t)y1,
                                      (int16_t)ox0, (int16_t)oy0, (int16_t)ox1, (int16_t)oy1};
                std::memcpy(R + 8 * k, r, sizeof(r));
                // LDS holds the needed columns widened to whole 4-byte quads
                // (+ 16: k_pyramid<true> reads a row's source window as three dwords, which
                // can reach 8 bytes past the last row's last quad)
                const int bytes = any ? 4 * ((x1 - (x0 & ~3) + 3) / 4) * (y1 - y0) : 0;
                int& buf = (k & 1) ? s.lds_b : s.lds_a;
                buf = std::max(buf, ((bytes + 15) & ~15) + 16);
                nx0 = x0; nx1 = x1; ny0 = y0; ny1 = y1;
            }
        }
    if (s.lds_a + s.lds_b > kPzMaxLds) { plan.why = "pyramid tile exceeds LDS (scale factor too large)"; return false; }
    return true;
}

static bool pyramid_tiles(Plan& plan) {
    const int L = plan.L;
    // debug builds: ORBX_PZ_TILE=WxH / ORBX_PZ_TILE2=WxH override the first / later
    // segments' tile size; switch pz_seg = n the levels per segment (0: one segment);
    // tuning, the output is the same
    int tw = kPzTW, th = kPzTH, tw2 = kPzTW2, th2 = kPzTH2, seg = kPzSegLevels;
    auto tile_env = [](const char* name, int& w, int& h) {
        int a = 0, b = 0;
        if (const char* e = debug_env(name))
            if (std::sscanf(e, "%dx%d", &a, &b) == 2 && a >= 16 && b >= 16) { w = a; h = b; }
    };
    tile_env("ORBX_PZ_TILE", tw, th);
    tile_env("ORBX_PZ_TILE2", tw2, th2);
    seg = tuning(Tune::PzSeg, seg);
    if (seg < 2 || seg > L) seg = L;
    plan.pz_nseg = 0;
    for (int l0 = 0;;) {
        PzSeg& s = plan.pz[plan.pz_nseg++];
        s = PzSeg{};
        s.l0 = l0;
        s.nl = std::min(seg, L - l0);
        if (!pyramid_segment(plan, s, l0 == 0 ? tw : tw2, l0 == 0 ? th : th2)) return false;
        if (l0 + s.nl >= L) break;
        l0 += s.nl - 1;
    }
    // k_pyramid<true> needs the source bytes of any 4 consecutive output columns (sx0 of the
    // first .. sx1 of the last) within 8 bytes: scale factors up to about 2
    // (switch pz_byte = 1 forces the byte-read form: tuning, the output is the same)
    plan.pz_win = tuning(Tune::PzByte, 0) <= 0;
    for (int l = 1; l < L && plan.pz_win; l++) {
        const LevelGeom& g = plan.lv[l];
        const int16_t* xt = plan.rtab.data() + g.xtab_off;
        for (int x = 0; x < g.w; x++)
            if (xt[4 * std::min(x + 3, g.w - 1) + 1] - xt[4 * x] > 7) { plan.pz_win = false; break; }
    }
    return true;
}

bool make_plan(Plan& plan, const OrbParams& prm, int W, int H) {
    plan = Plan();
    plan.prm = prm;
    plan.W = W;
    plan.H = H;
    plan.L = prm.nlevels;
    if (W <= 0 || H <= 0) { plan.why = "empty image"; return false; }
    long long off = 0;
    int cell_first = 0, key_off = 0, out_off = 0, tile_first = 0, slot_off = 0;
    int prev_w = W, prev_h = H;
    for (int l = 0; l < prm.nlevels; l++) {
        LevelGeom& g = plan.lv[l];
        std::memset(&g, 0, sizeof(g));
        const float s = prm.inv_scale[l];
        g.w = cv_roundf((float)W * s);                 // cc:1643
        g.h = cv_roundf((float)H * s);
        // below 33 px the reference's DistributeOctTree divides by a zero or negative
        // border-trimmed size (ORBextractor.cc:674-676: nIni = round(width / height),
        // vpIniNodes.resize(nIni)), so such frames are refused rather than given a meaning
        if (g.w < kMinLevelSide || g.h < kMinLevelSide) { plan.why = "pyramid level under 33 px"; return false; }
        if (g.w - 2 * kMinBorder >= 4096 || g.h - 2 * kMinBorder >= 4096) { plan.why = "frame too large"; return false; }
        g.pitch = (g.w + 63) & ~63;
        g.off = off;
        off += (long long)g.pitch * g.h;
        off = (off + 255) & ~255LL;
        g.scale = prm.scale[l];
        g.kp_size = (float)(int)(31 * prm.scale[l]);  // cc:1140
        g.N = prm.features[l];

        // FAST cell grid, cc:1025-1085
        const int minBorderX = kMinBorder, minBorderY = kMinBorder;
        const int maxBorderX = g.w - kEdge + 3, maxBorderY = g.h - kEdge + 3;
        const float width = (float)(maxBorderX - minBorderX);
        const float height = (float)(maxBorderY - minBorderY);
        const int nCols = (int)(width / 30.f);
        const int nRows = (int)(height / 30.f);
        // a level narrower or shorter than one 30-px FAST cell (under 62 px) has no cells:
        // the reference's cell loops run zero times and the level keeps no keypoints
        const bool no_cells = nCols <= 0 || nRows <= 0;
        const int wCell = no_cells ? 0 : (int)std::ceil(width / nCols);
        const int hCell = no_cells ? 0 : (int)std::ceil(height / nRows);
        g.cell_first = cell_first;
        g.key_off = key_off;
        int level_cap = 0;
        for (int i = 0; i < (no_cells ? 0 : nRows); i++) {
            const float iniY = (float)(minBorderY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(minBorderX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                CellGeom c{};
                c.level = l;
                c.x0 = (int)iniX;
                c.y0 = (int)iniY;
                c.cols = (int)maxX - c.x0;
                c.rows = (int)maxY - c.y0;
                const int wc = c.cols > 6 ? c.cols - 6 : 0, wr = c.rows > 6 ? c.rows - 6 : 0;
                if (wc > kCellMax || wr > kCellMax) { plan.why = "FAST cell wider than 64 px"; return false; }
                c.slot_off = slot_off;
                c.slot_cap = ((wc + 1) / 2) * ((wr + 1) / 2);
                c.pitch = g.pitch;
                plan.fc_wr = std::max(plan.fc_wr, wr);
                plan.fc_wc = std::max(plan.fc_wc, wc);
                c.src_off = (int)(g.off + (long long)(c.y0 + 3) * g.pitch + c.x0 + 3);
                slot_off += c.slot_cap;
                level_cap += c.slot_cap;
                plan.cells.push_back(c);
            }
        }
        g.ncells = (int)plan.cells.size() - cell_first;
        cell_first = (int)plan.cells.size();
        g.key_cap = level_cap;
        key_off += level_cap;
        if (level_cap > plan.max_key_cap) plan.max_key_cap = level_cap;

        // octree roots, cc:674-699
        const int minX = minBorderX, maxX = maxBorderX, minY = minBorderY, maxY = maxBorderY;
        g.nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
        // a level without keypoints never reads its root nodes (DistributeOctTree of no keys)
        if (level_cap == 0) g.nIni = std::min(std::max(g.nIni, 1), kMaxIni);
        if (g.nIni < 1 || g.nIni > kMaxIni) { plan.why = "aspect ratio outside octree support"; return false; }
        g.hX = (float)(maxX - minX) / g.nIni;
        for (int i = 0; i <= g.nIni; i++) g.ini_x0[i] = (int)(g.hX * (float)i);
        g.height_rel = maxY - minY;
        int ncap = g.N + 4;
        if (4 * g.nIni + 4 > ncap) ncap = 4 * g.nIni + 4;
        if (prm.node_cap_limit > 0 && prm.node_cap_limit < ncap) ncap = prm.node_cap_limit;
        g.ncap = ncap;
        g.out_off = out_off;
        out_off += ncap;
        if (ncap > plan.max_ncap) plan.max_ncap = ncap;

        // score/blur tiles (kLtTW x kLtTH outputs)
        g.tiles_x = (g.w + kLtTW - 1) / kLtTW;
        g.tiles_y = (g.h + kLtTH - 1) / kLtTH;
        g.tile_first = tile_first;
        tile_first += g.tiles_x * g.tiles_y;

        // resize tables
        if (l > 0) {
            g.xtab_off = (int)plan.rtab.size();
            plan.rtab.resize(plan.rtab.size() + 4 * (size_t)g.w);
            g.ytab_off = (int)plan.rtab.size();
            plan.rtab.resize(plan.rtab.size() + 4 * (size_t)g.h);
            resize_tables(prev_w, prev_h, g.w, g.h, plan.rtab.data() + g.xtab_off, plan.rtab.data() + g.ytab_off);
        }
        prev_w = g.w;
        prev_h = g.h;
    }
    if (!pyramid_tiles(plan)) return false;
    plan.pyr_frame_bytes = off;
    plan.slots_per_frame = slot_off;
    plan.keys_per_frame = key_off;
    plan.kept_per_frame = out_off;
    plan.tiles_total = tile_first;
    {
        // k_describe_tiles (switch desc_tiles = 1; measured slower than k_describe, DESIGN.md
        // section 4 item 5): k_octree bins each level's kept slots into its tiles with
        // NC-entry LDS counters and 16-bit list offsets
        const int NC = (plan.max_ncap + 63) & ~63;
        bool fits = true;
        for (int l = 0; l < plan.L; l++)
            fits = fits && plan.lv[l].tiles_x * plan.lv[l].tiles_y <= NC && plan.lv[l].ncap < 65536;
        plan.desc_tiles = fits && tuning(Tune::DescTiles, 0) == 1;
    }
    plan.rtab.resize(plan.rtab.size() + 64, 0);  // k_pyramid reads row taps in batches of 8 rows
    plan.ok = true;
    return true;
}

}  // namespace orbx
