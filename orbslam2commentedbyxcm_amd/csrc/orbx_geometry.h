// orbx_geometry.h -- host-side plan of one (params, W, H) extraction configuration.
//
// Everything that depends only on the ORB parameters and the frame size is computed
// once on the host, with the reference's exact float/double/int conversions, and
// uploaded as small tables: level sizes (ORBextractor.cc:1641-1643), the FAST cell
// grid (cc:1025-1085), octree root nodes (cc:674-699), resize coefficient tables
// (OpenCV 3.3.1 resize INTER_LINEAR), per-level budgets and scales (cc:438-500).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace orbx {

constexpr int kMaxLevels = 32;
constexpr int kMinLevelSide = 33;  // smallest pyramid level side make_plan accepts
constexpr int kEdge = 19;        // EDGE_THRESHOLD, ORBextractor.cc:46
constexpr int kMinBorder = 16;   // EDGE_THRESHOLD - 3, ORBextractor.cc:1032
constexpr int kMaxIni = 16;      // octree root nodes supported per level
constexpr int kCellMax = 64;     // max detection-window width/height of a FAST cell

#ifndef ORBX_LT_TH
#define ORBX_LT_TH 48
#endif
constexpr int kLtTW = 64, kLtTH = ORBX_LT_TH;  // k_level_tiles output tile (columns x rows)

// Parameters + derived per-level members (ORBextractor.h:204-219).
struct OrbParams {
    int nfeatures = 1000;
    double scale_factor = 1.2;   // double member, ORBextractor.h:207
    int nlevels = 8;
    int ini_th = 20;
    int min_th = 7;
    float scale[kMaxLevels], inv_scale[kMaxLevels], sigma2[kMaxLevels], inv_sigma2[kMaxLevels];
    int features[kMaxLevels];
    int umax[16];
    // orbx_extractor_set_node_capacity: > 0 lowers every level's octree node capacity
    // below the bound the reference's algorithm guarantees (max(N+4, 4 nIni+4)), which
    // makes the kernels' overflow status observable in tests.  0 = the guaranteed bound.
    int node_cap_limit = 0;
};
bool init_params(OrbParams& p, int nfeatures, float scale_factor, int nlevels, int ini, int min);

// One level of one frame, as laid out on the device.
struct LevelGeom {
    int w, h;              // ROI size
    int pitch;             // row pitch (bytes) of this level in the pyramid/blur buffers
    int pad0;
    long long off;         // byte offset of the level inside one frame's pyramid block
    // FAST cells
    int cell_first, ncells;
    // candidates (per-frame key region)
    int key_off, key_cap;
    // octree
    int N;                 // mnFeaturesPerLevel[level]
    int nIni;
    float hX;
    int ncap;              // node capacity = max kept keypoints
    int out_off;           // offset of this level's kept slots in a frame's kept array
    int ini_x0[kMaxIni + 1];  // root node x boundaries: node i = [ini_x0[i], ini_x0[i+1])
    int height_rel;        // maxY - minY (root node bottom)
    // output
    float scale;           // mvScaleFactor[level]
    float kp_size;         // (float)(int)(PATCH_SIZE * scale)
    // blur tiles
    int tile_first, tiles_x, tiles_y;
    // resize tables (levels >= 1)
    int xtab_off, ytab_off;  // offsets (in int16 units) into the resize table buffer
};

// One FAST cell: sub-image [y0, y0+rows) x [x0, x0+cols) of its level ROI.
struct CellGeom {
    int level;
    int x0, y0, cols, rows;
    int slot_off;          // offset of this cell's candidate slots in the frame's slot array
    int slot_cap;
    int src_off;           // level.off + (y0 + 3) * pitch + x0 + 3: detection window origin in a frame block
    int pitch;             // level row pitch
};

// k_pyramid: one workgroup per (frame, tile) computes every level of its tile.  A
// tile owns a rectangle of every level (kPzTW x kPzTH at level 0, boundaries carried up
// the cascade by the resize tables); its "needed" rectangle at level l is what it owns
// plus the source footprint of its needed rectangle at level l + 1, so levels chain
// inside LDS with a small recomputed right / bottom halo.  Per (tile, level) the table
// holds 8 int16: needed x0, y0, x1, y1 and owned x0, y0, x1, y1 (ends exclusive).
// Deep pyramids are built in segments of at most kPzSegLevels levels, one launch each:
// a segment after the first takes its input level (the previous segment's last, already
// in HBM) as its "level 0" and owns none of it.  Each segment's halo then grows over at
// most kPzSegLevels - 1 resizes instead of L - 1 (12 levels: ~32 px of recomputed
// right / bottom halo per 128 x 96 level-0 tile and 35 KB of LDS, against ~13 px and
// 27 KB for 8), at the price of re-reading one small level.  Later segments tile their
// input level by kPzTW2 x kPzTH2.
constexpr int kPzTW = 128, kPzTH = 96;
constexpr int kPzTW2 = 64, kPzTH2 = 48;
constexpr int kPzSegLevels = 8;
constexpr int kPzMaxSegs = kMaxLevels;
constexpr int kPzMaxLds = 150 * 1024;

struct PzSeg {
    int l0 = 0, nl = 0;           // input level and level count (l0 .. l0 + nl - 1)
    int nx = 0, ny = 0, tiles = 0;  // tile grid over level l0
    int off = 0;                  // offset (int16 units) of the tile rectangles in rtab
    int lds_a = 0, lds_b = 0;     // LDS ping / pong buffers (even / odd levels of the segment), bytes
};

struct Plan {
    int W = 0, H = 0, L = 0;
    OrbParams prm;
    LevelGeom lv[kMaxLevels];
    std::vector<CellGeom> cells;
    std::vector<int16_t> rtab;      // resize tables: per level xtab (w*4) then ytab (h*4)
    long long pyr_frame_bytes = 0;  // one frame's pyramid block (levels 0..L-1)
    int slots_per_frame = 0;        // candidate slots per frame (sum of cell caps)
    int keys_per_frame = 0;         // candidate key capacity per frame
    int kept_per_frame = 0;         // sum of ncap
    int tiles_total = 0;            // blur tiles per frame
    int pz_nseg = 0;                // k_pyramid segments (launches)
    PzSeg pz[kPzMaxSegs];
    bool pz_win = false;            // k_pyramid<true>: every 4 columns' resize taps span <= 8 source bytes
    int fc_wr = 0, fc_wc = 0;       // largest FAST detection window (rows, cols)
    int max_ncap = 0;
    // describe in level-tile order (k_describe_tiles, bins from k_octree) instead of
    // keypoint by keypoint: ORBX_DESC_TILES=1, when every level's tiles fit the octree's
    // NC-entry LDS arrays (a measured alternative, slower at configs[1] and [4])
    bool desc_tiles = false;
    int max_key_cap = 0;
    bool ok = false;
    const char* why = nullptr;
};

bool make_plan(Plan& plan, const OrbParams& prm, int W, int H);

}  // namespace orbx
