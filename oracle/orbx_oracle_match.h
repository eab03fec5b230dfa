/* orbx_oracle_match.h -- TEST INFRASTRUCTURE ONLY: CPU restatement of the matching
 * functions (see orbx_oracle_match.c).  Parity status: "parity unpinned" against the
 * reference binary (OpenCV/Eigen-dependent reference cannot be built here). */
#ifndef ORBX_ORACLE_MATCH_H
#define ORBX_ORACLE_MATCH_H

#include <stdint.h>

#include "orbx_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORA_GRID_COLS 64 /* FRAME_GRID_COLS, Frame.h:37 */
#define ORA_GRID_ROWS 48 /* FRAME_GRID_ROWS, Frame.h:38 */

/* The Frame / KeyFrame fields the matchers read (Frame.h). */
typedef struct {
    int n;                     /* N */
    const ora_keypoint* keys;  /* mvKeysUn */
    const uint8_t* desc;       /* mDescriptors, n x 32 */
    const float* u_right;      /* mvuRight or NULL */
    float fx, fy, cx, cy, bf, b;
    float min_x, max_x, min_y, max_y; /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    int nlevels;
    const float* scale_factors;  /* mvScaleFactors */
    const float* level_sigma2;   /* mvLevelSigma2 */
    float Tcw[12];               /* mTcw rows 0..2, row-major */
} ora_frame;

typedef struct {
    float inv_w, inv_h;
    int start[ORA_GRID_COLS * ORA_GRID_ROWS + 1]; /* cell c = ix*ROWS + iy */
    int* idx;
} ora_grid;

typedef struct {
    int n;
    const float* pos;            /* GetWorldPos(), n x 3 */
    const uint8_t* desc;         /* GetDescriptor(), n x 32 */
    const int32_t* observations; /* Observations() */
    const uint8_t* bad;          /* isBad() or NULL */
    const float* max_distance;   /* mfMaxDistance */
    const float* min_distance;   /* mfMinDistance */
    const float* normal;         /* GetNormal(), n x 3 */
} ora_mappoints;

/* Frame::IsInFrustum outputs per MapPoint (Frame.cc:412-477) */
typedef struct {
    const uint8_t* in_view;     /* mbTrackInView */
    const float* proj_x;        /* mTrackProjX */
    const float* proj_y;        /* mTrackProjY */
    const float* proj_xr;       /* mTrackProjXR */
    const int32_t* scale_level; /* mnTrackScaleLevel */
    const float* view_cos;      /* mTrackViewCos */
} ora_track;

void ora_grid_build(const ora_frame* f, ora_grid* g);
void ora_grid_free(ora_grid* g);
int ora_features_in_area(const ora_frame* f, const ora_grid* g, float x, float y, float r, int minLevel, int maxLevel,
                         int* out, int cap);
void ora_compute_three_maxima(const int* histo_sizes, int L, int* ind1, int* ind2, int* ind3);
int ora_sbp_local(const ora_frame* f, int32_t* frame_mp, const int32_t* queries, int nq, const ora_mappoints* mps,
                  const ora_track* trk, float th, float nnratio);
void ora_is_in_frustum(const ora_frame* f, const ora_mappoints* mps, const int32_t* ids, int n,
                       float viewingCosLimit, uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                       int32_t* scale_level, float* view_cos);
void ora_create_mappoints(const ora_frame* f, const float* depth, float const_depth, float* pos, float* normal,
                          float* max_distance, float* min_distance, uint8_t* valid);
/* Tracking::UpdateLastFrame (Tracking.cc:893-954): temporal MapPoints of a stereo LastFrame */
int ora_update_last_frame(const ora_frame* f, const float* depth, float th_depth, int32_t* mp_obs, float* pos);
int ora_sbp_frame(const ora_frame* cur, int32_t* cur_mp, const ora_frame* last, const int32_t* last_mp,
                  const uint8_t* last_outlier, const ora_mappoints* mps, float th, int bMono, int check_ori);
int ora_sbp_keyframe(const ora_frame* cur, int32_t* cur_mp, const ora_frame* kf, const int32_t* kf_mp,
                     const uint8_t* already_found, const ora_mappoints* mps, float th, int orb_dist, int check_ori);
int ora_sbp_sim3(const ora_frame* kf, const float* Scw, const int32_t* points, int npoints, int32_t* matched,
                 const ora_mappoints* mps, int th);
int ora_search_for_triangulation(const ora_frame* kf1, const uint8_t* kf1_has_mp, const int32_t* fv1_node,
                                 const int32_t* fv1_off, const int32_t* fv1_idx, int fv1_n, const ora_frame* kf2,
                                 const uint8_t* kf2_has_mp, const int32_t* fv2_node, const int32_t* fv2_off,
                                 const int32_t* fv2_idx, int fv2_n, const float* F12, int bOnlyStereo, int check_ori,
                                 int32_t* pairs);
int ora_search_by_bow_kf_frame(const ora_frame* kf, const int32_t* kf_mp, const int32_t* fv1_node,
                               const int32_t* fv1_off, const int32_t* fv1_idx, int fv1_n, const ora_frame* f,
                               const int32_t* fv2_node, const int32_t* fv2_off, const int32_t* fv2_idx, int fv2_n,
                               float nnratio, int check_ori, int32_t* matches);
int ora_search_by_bow_kf_kf(const ora_frame* kf1, const int32_t* mp1, const int32_t* fv1_node, const int32_t* fv1_off,
                            const int32_t* fv1_idx, int fv1_n, const ora_frame* kf2, const int32_t* mp2,
                            const int32_t* fv2_node, const int32_t* fv2_off, const int32_t* fv2_idx, int fv2_n,
                            float nnratio, int check_ori, int32_t* matches12);
int ora_search_for_initialization(const ora_frame* f1, const ora_frame* f2, float* prev_matched, int32_t* matches12,
                                  int windowSize, float nnratio, int check_ori);
void ora_fuse(const ora_frame* kf, const int32_t* points, int npoints, const uint8_t* skip, const ora_mappoints* mps,
              float th, int32_t* best);
void ora_fuse_sim3(const ora_frame* kf, const float* Scw, const int32_t* points, int npoints, const uint8_t* skip,
                   const ora_mappoints* mps, float th, int32_t* best);
int ora_search_by_sim3(const ora_frame* kf1, const int32_t* mp1, const uint8_t* already1, const ora_frame* kf2,
                       const int32_t* mp2, const uint8_t* already2, const ora_mappoints* mps, float s12,
                       const float* R12, const float* t12, float th, int32_t* matches12);
void ora_distinctive_descriptors(int nmp, const int32_t* off, const uint8_t* desc, int32_t* best);
void ora_undistort_points(const float* K, const float* D, const float* pts, int n, float* out);
void ora_compute_stereo_matches(const ora_frame* left, const ora_keypoint* keys_r, const uint8_t* desc_r, int nr,
                                const uint8_t* const* levels_l, const uint8_t* const* levels_r, const int* level_w,
                                const int* level_h, const float* inv_scale, float maxD, float* u_right, float* depth);

/* Frame::ComputeStereoFromRGBD (Frame.cc:888-909) after Tracking::GrabImageRGBD's
 * convertTo(CV_32F, mDepthMapFactor) (Tracking.cc:265-271). */
void ora_compute_stereo_from_rgbd(const ora_keypoint* keys, const ora_keypoint* keys_un, int n, const void* depth,
                                  int depth_f32, int width, int height, long long row_bytes, float depth_map_factor,
                                  float bf, float* u_right, float* out_depth);
/* Tracking::TrackWithMotionModel's search (Tracking.cc:975-994): SearchByProjection at th,
 * again at 2*th from an empty mvpMapPoints when it found fewer than 20 matches. */
int ora_track_motion_model(const ora_frame* cur, int32_t* cur_mp, const ora_frame* last, const int32_t* last_mp,
                           const uint8_t* last_outlier, const ora_mappoints* mps, float th, int bMono, int check_ori,
                           int* retried);

/* H4: 1 (default) = the reference build's fused projection / epipolar forms, 0 = unfused */
void ora_set_match_contract_mode(int mode);

#ifdef __cplusplus
}
#endif
#endif
