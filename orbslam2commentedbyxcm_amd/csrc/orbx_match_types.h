// orbx_match_types.h -- device-side records of the projection-search matcher.
//
// One "problem" = one ORBmatcher::SearchByProjection call: the keypoints of the frame
// being searched (mvKeysUn, mDescriptors, mvuRight, mvpMapPoints) and the ordered
// list of projected queries (MapPoints).  Shared by host and device code.
#pragma once

#include <cstdint>

#include "orbx.h"

namespace orbx {

constexpr int kGridCols = 64;  // FRAME_GRID_COLS, Frame.h:37
constexpr int kGridRows = 48;  // FRAME_GRID_ROWS, Frame.h:38
constexpr int kHistoLength = 30;  // ORBmatcher::HISTO_LENGTH, ORBmatcher.cc:40

// One projected MapPoint, in the reference's iteration order.
struct ProjQuery {
    float u, v;           // window centre (projection)
    float ur;             // projected right-image u (stereo check)
    float r;              // GetFeaturesInArea radius
    float er_max;         // reject if |ur - mvuRight| > er_max where mvuRight > 0; < 0 = no check
    int min_level, max_level;  // GetFeaturesInArea level arguments
    int post_min, post_max;    // extra candidate level filter [post_min, post_max] (post_max < 0 = none)
    int mp;               // MapPoint id written to mvpMapPoints on a match; < 0 = skip query
    float angle;          // keypoint angle of the query (rotation histogram)
    int pad;              // 48-byte record
};

struct ProjProblem {
    const orbx_keypoint* keys;  // n keypoints of the searched frame (mvKeysUn)
    const uint8_t* desc;        // n x 32
    const float* u_right;       // n or null
    int32_t* frame_mp;          // n, in/out: mvpMapPoints as MapPoint ids, -1 = NULL
    int n;
    const ProjQuery* q;         // nq queries
    const uint8_t* qdesc;       // nq x 32 MapPoint descriptors
    int nq;
    float min_x, min_y, inv_w, inv_h;  // mnMinX, mnMinY, mfGridElementWidthInv/HeightInv
    int32_t* nmatches;          // out
};

// Global scratch per query (u64 words) when the per-query state does not fit in LDS.
#ifndef ORBX_TOPK
// candidate-list length per query (build constant, a multiple of 4).  12 measured
// configs[4] 86.6k frames/s against 81.5k for 8 and 85.0k for 16 (a list that runs out
// is re-scored on the replay's critical path), configs[1] within noise
// (profiles/r02_n_topk_ab.log)
#define ORBX_TOPK 12
#endif
// the candidate list (ORBX_TOPK u32) + mp, angle, match list, bin
constexpr int kProjScratchWords = ORBX_TOPK / 2 + 2;

#ifndef ORBX_SCORE_COUNT
#define ORBX_SCORE_COUNT 0  // diagnostics build: the scoring loop's visit counts in stamp words 17-22
#endif
// ProjParams::stamps words per problem.  The replay forms use words 9, 14 and 15
// differently, so word kStampForm records which one wrote them: 64 for the one-wave replay
// (9 = chunk loads + first rounds, a clock reading in 15), the replay's thread count for the
// block replay (9 = rounds, 14 = chunk loads, 15 = commits: durations).
constexpr int kStampForm = 16;
constexpr int kStampScore = 17;
constexpr int kStampWords = ORBX_SCORE_COUNT ? 23 : 17;

// Call-level semantics of the SearchByProjection overload being executed.
struct ProjParams {
    const int32_t* mp_obs;  // Observations() per MapPoint id (blocked_mode 0)
    int blocked_mode;       // 0: skip kp if mvpMapPoints[i] && ->Observations() > 0 (a11, a12)
                            // 1: skip kp if mvpMapPoints[i] (a13, a14)
    int accept_th;          // best distance threshold (<=): TH_HIGH, ORBdist or TH_LOW
    int ratio_mode;         // 1: reject if bestLevel==bestLevel2 && best > nnratio*second (a11)
    float nnratio;
    int check_ori;          // rotation-consistency histogram (a12, a13)
    unsigned long long* stamps;  // optional: kStampWords per-problem phase stamps and counters (diagnostics)
    int noct;               // octave buckets of the sorted grid: > every keypoint octave (1..32)
    int32_t* out_mp;        // optional (k_seq_commit): mvpMapPoints written here instead of
                            // frame_mp -- host-mapped memory for the single host calls
};

// Batched frame-to-frame matching over an extracted device sequence.
struct SeqArgs {
    const orbx_keypoint* kps;  // [B][cap]
    const uint8_t* desc;       // [B][cap][32]
    const int32_t* n;          // [B]
    int cap;
    const float* Tcw;          // [B][12]
    const float* u_right;      // [B][cap] mvuRight or null (monocular)
    const float* mp_pos;       // [B][cap][3] world position of keypoint i's MapPoint, or null: depth model
    const uint8_t* has_mp;     // [B][cap] LastFrame keypoint has a (non-outlier) MapPoint, or null: all
    float fx, fy, cx, cy, bf, b;
    float min_x, max_x, min_y, max_y;
    float depth;               // depth model: MapPoint depth along the last frame's rays
    int mono;                  // bMono
    int global_ids;            // MapPoint ids written: 0 = LastFrame keypoint index i, 1 = (b-1)*cap + i
    float th;                  // search radius factor
    float scale[32];           // mvScaleFactors
    int32_t* cur_mp;           // [B][cap] out (pre-filled -1)
    int32_t* nmatches;         // [B] out
    int retry_below;           // 0: the first search; > 0: the retry pass over the pairs with fewer matches
};

// Tracking::SearchLocalPoints over a batch of Frames (orbx_search_local_points_device):
// Frame::IsInFrustum of every local MapPoint, then SearchByProjection(Frame&, vector<MapPoint*>, th).
struct LocalArgs {
    const orbx_keypoint* kps;  // [B][cap] mvKeysUn
    const uint8_t* desc;       // [B][cap][32]
    const int32_t* n;          // [B]
    const float* u_right;      // [B][cap] or null
    int cap;
    const float* Tcw;          // [B][12]
    float fx, fy, cx, cy, bf;
    float min_x, max_x, min_y, max_y;
    float scale[32];           // mvScaleFactors
    int nlevels;
    float log_scale;           // mfLogScaleFactor = (float)log(mfScaleFactor)
    int nmp;                   // MapPoint table
    const float* pos;          // [nmp][3]
    const uint8_t* mdesc;      // [nmp][32]
    const float* normal;       // [nmp][3]
    const float* max_distance; // [nmp] mfMaxDistance
    const float* min_distance; // [nmp] mfMinDistance
    const uint8_t* bad;        // [nmp] or null
    const int32_t* local_off;  // [B+1] frame b's local map = local_ids[local_off[b] .. local_off[b+1])
    const int32_t* local_ids;
    float th;                  // SearchByProjection th
    float cos_limit;           // IsInFrustum viewingCosLimit
    int32_t* frame_mp;         // [B][cap] in/out: mvpMapPoints as MapPoint ids
    int32_t* nmatches;         // [B] out
    int hash_size;             // LDS hash slots (power of two >= 2 cap)
};

// SearchForTriangulation: one unmatched KF1 keypoint of a shared vocabulary node.
struct TriQuery {
    int idx1;       // KF1 keypoint
    int beg, end;   // its node's KF2 keypoints: fv2_idx[beg..end)
    int stereo1;    // mvuRight[idx1] >= 0
};

struct TriProblem {
    const orbx_keypoint* keys1;
    const uint8_t* desc1;
    const orbx_keypoint* keys2;
    const uint8_t* desc2;
    const float* u_right2;      // or null
    const uint8_t* has_mp2;     // KF2 keypoint already has a MapPoint
    const int32_t* fv2_idx;
    const float* scale2;        // KF2 mvScaleFactors
    const float* sigma2_2;      // KF2 mvLevelSigma2
    float F12[9];
    float ex, ey;               // epipole of KF1's centre in KF2
    int only_stereo;
    int check_ori;
    int n2;
    const TriQuery* q;
    int nq;
    int32_t* matches12;         // out: vMatches12 (KF1 n), pre-filled with -1
    long long scratch_off;
    int n1;                     // KF1 keypoints (read by the pair compaction only)
    int32_t* pairs_out;         // or null: vMatchedPairs (idx1, idx2) in idx1 order
    int32_t* npairs_out;        // its count
};

// Batched SearchForTriangulation (orbx_search_for_triangulation_batch_device): one
// keyframe's device arrays (orbx_keyframe_device without the host pose) ...
struct TriKF {
    const orbx_keypoint* keys;
    const uint8_t* desc;
    const int32_t* n;
    const float* u_right;
    const uint8_t* has_mp;
    const int32_t* fv_node;
    const int32_t* fv_off;
    const int32_t* fv_idx;
    const int32_t* nfv;
};

// ... and one (KF1, KF2) pair with the host-side quantities of the reference's loop
// (F12 from LocalMapping::ComputeF12, the epipole of ORBmatcher.cc:858-865).
struct TriPair {
    int kf1, kf2;
    float F12[9];
    float ex, ey;
};

struct TriBatch {
    const TriKF* kfs;
    const TriPair* pairs;
    int npairs;
    int cap;
    int only_stereo;
    int check_ori;
    const float* scale2;        // mvScaleFactors (shared camera)
    const float* sigma2_2;      // mvLevelSigma2
    TriQuery* q;                // [P][cap]
    TriProblem* probs;          // [P]
    int32_t* matches12;         // [P][cap]
    int32_t* pairs_out;         // [P][cap][2]
    int32_t* npairs_out;        // [P]
};

// SearchByBoW (KF->F and KF->KF): one shared vocabulary node.  Its queries (side-1
// keypoints with a valid MapPoint, node-list order) are q_idx1[q_beg..q_end); its
// side-2 candidates are fv2_idx[c_beg..c_end) (ascending index, the node list).
struct BowNode {
    int q_beg, q_end;
    int c_beg, c_end;
};

struct BowProblem {
    const uint8_t* desc1;
    const orbx_keypoint* keys1;
    const uint8_t* desc2;
    const orbx_keypoint* keys2;
    const int32_t* q_idx1;      // queries (side-1 keypoint indices), node by node
    const int32_t* fv2_idx;     // side-2 FeatureVector indices
    const uint8_t* avail2;      // side-2 keypoint may be matched (KF->KF: has a good MapPoint)
    const int32_t* mp1;         // side-1 MapPoint ids (KF->F: written to the frame)
    const int32_t* mp2;         // side-2 MapPoint ids (KF->KF: written to matches12)
    const BowNode* nodes;
    int nnodes;
    int n1, n2;
    int kf_kf;                  // 0: SearchByBoW(KF, F) (accept <= TH_LOW); 1: (KF, KF) (accept < TH_LOW)
    float nnratio;
    int check_ori;
    int32_t* matches;           // KF->F: [n2] frame matches; KF->KF: [n1] matches12 (pre-filled -1)
};

// SearchForInitialization: F2's grid (Frame::mGrid as CSR) and the level-0 queries of F1.
struct InitProblem {
    const orbx_keypoint* keys1;
    const uint8_t* desc1;
    const orbx_keypoint* keys2;
    const uint8_t* desc2;
    const int32_t* cell_start;  // [kNumCells + 1], cell c = ix * FRAME_GRID_ROWS + iy
    const int32_t* cell_idx;    // keypoint indices, ascending within a cell
    const int32_t* q_idx1;      // F1 keypoints with octave 0, ascending
    const float* prev;          // vbPrevMatched [n1][2]
    int nq, n1, n2;
    float min_x, min_y, inv_w, inv_h;
    float r;                    // windowSize
    float nnratio;
    int check_ori;
    int32_t* matches12;         // out [n1] (vnMatches12)
    unsigned long long* lists;  // scratch [nq][8]
    int* trunc;                 // scratch [nq]
};

// Fuse / SearchBySim3: one projected MapPoint searched in a keyframe's grid window
// for the first keypoint with the smallest distance (no claims).
struct BestQuery {
    float u, v, ur, r;  // projection, right-image u (Fuse gate), GetFeaturesInArea radius
    int pred;           // predicted level: candidates with octave in [pred-1, pred]
    int pad[3];         // 32-byte record
};

struct BestProblem {
    const orbx_keypoint* keys;  // searched keyframe (mvKeysUn)
    const uint8_t* desc;
    const float* u_right;       // mvuRight or null (gate only)
    const int32_t* cell_start;  // mGrid as CSR, cell c = ix * FRAME_GRID_ROWS + iy
    const int32_t* cell_idx;
    float inv_sigma2[32];       // mvInvLevelSigma2 (gate only)
    float min_x, min_y, inv_w, inv_h;
    const BestQuery* q;
    const uint8_t* qdesc;       // nq x 32
    int nq;
    int gate;                   // 1: Fuse(KF, vpMapPoints) chi-square gate (5.99 mono / 7.8 stereo)
    int accept;                 // best distance threshold (<=)
    int32_t* best;              // out [nq]: keypoint index or -1
};

struct StereoResult {
    int reach_sort;  // the iteration reaches the in-loop outlier pass (no `continue`)
    int pushed;      // (dist, iL) was appended to vDistIdx
    int dist;        // SAD distance pushed
    float u_right;
    float depth;
};

// Frame::ComputeStereoMatches (Frame.cc:673-885) over B left/right pairs: pair b's left
// keypoints keys_l[b*cap ...] (min(n_l[b], cap) of them), right keypoints keys_r[b*cap
// ...], pyramid levels of the left / right extractor at pyr_l + b*fb_l / pyr_r + b*fb_r.
struct StereoBatch {
    const orbx_keypoint* keys_l;  // mvKeys
    const uint8_t* desc_l;        // mDescriptors
    const int32_t* n_l;
    const orbx_keypoint* keys_r;  // mvKeysRight
    const uint8_t* desc_r;        // mDescriptorsRight
    const int32_t* n_r;
    int cap;                      // keypoint slots per frame
    int rows;                     // vRowIndices size: mvImagePyramid[0].rows
    int nlevels;                  // octaves of the keypoints (mvScaleFactors entries)
    int band_cap;                 // row_idx slots per pair (= cap: every right keypoint once)
    // vRowIndices, restated: the right keypoints as a CSR over (octave, floor(y)) --
    // row_off[b][o * rows + y] .. [+1] into row_idx[b] -- then rows words: how many right
    // keypoints' bands [floor(y - r), ceil(y + r)] cover each image row (the reference's
    // vRowIndices[row].size(), whose emptiness decides whether a left keypoint is searched)
    int32_t* row_off;             // [B][nlevels * rows + 1 + rows]
    int32_t* row_idx;             // [B][band_cap]
    const uint8_t* pyr_l;         // mvImagePyramid ROIs of the left / right extractor
    const uint8_t* pyr_r;
    long long fb_l, fb_r;         // pyramid bytes per frame
    // level 0 read in place by the extraction (orbx_extractor_set_level0_in_place): pair b's
    // level 0 is the caller's frame at l0_* + b * l0_fp_*, rows l0_pitch_* apart (null: in pyr_*)
    const uint8_t* l0_l;
    const uint8_t* l0_r;
    long long l0_fp_l, l0_fp_r;
    int l0_pitch_l, l0_pitch_r;
    long long level_off[32];      // level l of a frame block at + level_off[l], rows level_pitch[l] apart
    int level_pitch[32];
    int level_w[32];
    float scale[32];              // mvScaleFactors
    float inv_scale[32];          // mvInvScaleFactors
    float bf;                     // mbf
    float max_d;                  // maxD = mbf / minZ
    StereoResult* res;            // [B][cap] per-keypoint results before the outlier pass
    float* u_right;               // [B][cap] out: mvuRight (-1 = none; slots >= n_l[b] too)
    float* depth;                 // [B][cap] out: mvDepth
};



}  // namespace orbx
