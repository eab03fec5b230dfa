/*
 * orbx.h -- C ABI of the MI355X-native ORB extraction + Hamming matching library
 * (liborbx.so, built from orbslam2commentedbyxcm_amd/csrc/).
 *
 * This is the drop-in boundary for ORB-SLAM2's per-frame hot path.  Every entry
 * point names the reference interface it replaces (paths relative to the
 * reference repository, xcmworkharder/OrbSlam2CommentedByXcm):
 *
 *   ORBextractor::ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
 *       include/ORBextractor.h:93, src/ORBextractor.cc:438-550  -> orbx_extractor_create
 *   ORBextractor::operator()(image, mask, keypoints, descriptors)
 *       include/ORBextractor.h:111, src/ORBextractor.cc:1513-1629 -> orbx_extract,
 *       orbx_extract_batch, orbx_extract_batch_device
 *   ORBextractor::Get{Levels,ScaleFactor,ScaleFactors,InverseScaleFactors,
 *       ScaleSigmaSquares,InverseScaleSigmaSquares}
 *       include/ORBextractor.h:119-159                              -> orbx_extractor_levels
 *   ORBextractor::mvImagePyramid (public member read by Frame::ComputeStereoMatches)
 *       include/ORBextractor.h:162, src/Frame.cc:682,782,810,816    -> orbx_pyramid_level
 *   ORBmatcher::DescriptorDistance(a, b)
 *       include/ORBmatcher.h:65, src/ORBmatcher.cc:1983-2003        -> orbx_hamming,
 *       orbx_hamming_matrix_device
 *   ORBmatcher candidate scoring inside SearchByProjection / SearchForTriangulation
 *       src/ORBmatcher.cc:61-173, 1620-1789, 1792-1924, 850-1056     -> orbx_window_match
 *
 * Conventions: every function returns an int status (ORBX_OK = 0, ORBX_EMPTY = 1
 * for the reference's silent empty-image no-op, negative on error) and never
 * throws.  All pointers are plain host or device pointers; no C++ or torch types
 * cross this boundary.  One extractor owns one HIP stream and is not re-entrant
 * (like the reference's stateful ORBextractor); distinct extractors may be used
 * from distinct threads concurrently (Frame.cc:127-131).
 */
#ifndef ORBX_H
#define ORBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORBX_OK 0
#define ORBX_EMPTY 1
#define ORBX_ERR_ARG -1
#define ORBX_ERR_HIP -2
#define ORBX_ERR_CAPACITY -3
#define ORBX_ERR_UNSUPPORTED -4
#define ORBX_ERR_STATE -5

#define ORBX_MAX_LEVELS 32

/* Binary-identical to cv::KeyPoint {Point2f pt; float size, angle, response; int octave, class_id;} */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbx_keypoint;

/* The five YAML parameters of Tracking.cc:129-149 (ORBextractor.{nFeatures,scaleFactor,
 * nLevels,iniThFAST,minThFAST}). */
typedef struct {
    int nfeatures;
    float scale_factor;
    int nlevels;
    int ini_th_fast;
    int min_th_fast;
} orbx_extractor_params;

typedef struct orbx_extractor orbx_extractor;

/* ORBextractor::ORBextractor.  Selects HIP device `device`, creates one stream. */
int orbx_extractor_create(const orbx_extractor_params* params, int device, orbx_extractor** out);
void orbx_extractor_destroy(orbx_extractor* ex);

/* GetLevels/GetScaleFactors/...: each non-null array receives nlevels floats. */
int orbx_extractor_levels(const orbx_extractor* ex, int* nlevels, float* scale, float* inv_scale,
                          float* sigma2, float* inv_sigma2);
/* mnFeaturesPerLevel (ORBextractor.h:212): nlevels ints. */
int orbx_extractor_features_per_level(const orbx_extractor* ex, int* features);

/* Upper bound on keypoints one W x H frame can produce (size `cap` with it). */
int orbx_extractor_max_keypoints(orbx_extractor* ex, int width, int height, int* max_kps);

/* ORBextractor::operator() on one host image (row stride in bytes).  Keypoints in
 * the reference order (level-major, octree-list order), coordinates scaled to level
 * 0; descriptors n x 32 bytes.  Returns ORBX_EMPTY (outputs untouched) for an empty
 * image, ORBX_ERR_CAPACITY if more than `cap` keypoints were found (*n_out then
 * holds the required count).  Frame size: pyramid levels under 62 px on a side hold no
 * FAST cell and keep no keypoints, as in the reference (ORBextractor.cc:1047-1085); a
 * frame with a level under 33 px returns ORBX_ERR_UNSUPPORTED (the reference's
 * DistributeOctTree divides by a zero or negative size there, cc:674-676), as do
 * levels over 4096 px and aspect ratios beyond 16 octree roots. */
int orbx_extract(orbx_extractor* ex, const uint8_t* img, int width, int height, size_t stride,
                 orbx_keypoint* kps, uint8_t* desc, int cap, int* n_out);

/* Wall time (microseconds) of the newest orbx_extract / orbx_extract_batch host call on
 * `ex`, entry to return: what a C++ caller pays per call (diagnostics; -1 for NULL). */
double orbx_extractor_last_call_us(const orbx_extractor* ex);

/* The same for B host images of one size; frame b writes kps[b*cap ...],
 * desc[b*cap*32 ...] and n_per_frame[b]. */
int orbx_extract_batch(orbx_extractor* ex, int batch, const uint8_t* const* imgs, int width,
                       int height, size_t stride, orbx_keypoint* kps, uint8_t* desc, int cap,
                       int* n_per_frame);

/* Device-resident fast path: d_imgs holds B frames (frame b at d_imgs + b*frame_pitch,
 * rows `stride` bytes apart) already in HBM; outputs are device pointers as above.
 * Work is enqueued on the extractor's stream (or on `stream` if non-null, a
 * hipStream_t) and the call returns without synchronising.  n_per_frame[b] receives
 * the full count even when it exceeds cap (only cap keypoints are then written). */
int orbx_extract_batch_device(orbx_extractor* ex, int batch, const uint8_t* d_imgs,
                              size_t frame_pitch, int width, int height, size_t stride,
                              orbx_keypoint* d_kps, uint8_t* d_desc, int cap, int* d_n_per_frame,
                              void* stream);

/* The extractor's hipStream_t (as void*). */
void* orbx_extractor_stream(orbx_extractor* ex);

/* Scheduling hook for running other work beside a batched extraction (no reference
 * counterpart): from now on every extraction records `*event` (a hipEvent_t owned by the
 * extractor) on its stream right after stage `stage` -- 1 pyramid, 2 blur + FAST
 * strength, 3 FAST cells, 4 octree; 0 stops recording.  orbx_stream_wait_event makes
 * another stream wait for the latest record (hipStreamWaitEvent). */
int orbx_extractor_set_stage_event(orbx_extractor* ex, int stage, void** event);
int orbx_stream_wait_event(void* stream, void* event);

/* A HIP stream on `device`.  cu_stride k > 1: its kernels run only on compute units 0,
 * k, 2k, ... (hipExtStreamCreateWithCUMask: default priority, and a blocking stream --
 * it synchronises with the null stream, so a caller that issues null-stream work beside
 * it serialises against it); otherwise a non-blocking stream from
 * hipStreamCreateWithPriority with `priority` (HIP's range: lower numbers are higher
 * priorities; 0 = default).  The batched front end creates its matcher
 * stream with it before the extraction lanes' streams, so that the three busy streams
 * get hardware queues of their own.  No reference counterpart:
 * ORB-SLAM2 tracks one frame at a time.  Release with orbx_stream_destroy. */
int orbx_stream_create(int device, int cu_stride, int priority, void** stream);
int orbx_stream_destroy(void* stream);

/* Kernel status of the last extraction (any path), per frame: 0 = complete; bit 0
 * (ORBX_STATUS_NODE_OVERFLOW) = an octree level needed more nodes than its capacity
 * (or held more than 65535 FAST keypoints, the octree's u16 counters),
 * bit 1 (ORBX_STATUS_ITERATIONS) = an octree loop hit its iteration guard; either way
 * that frame's keypoints are truncated and differ from the reference's DistributeOctTree
 * (ORBextractor.cc:667-1013).  The host paths (orbx_extract, orbx_extract_batch) turn a
 * non-zero status into ORBX_ERR_STATE; orbx_extract_batch_device returns before the
 * kernels run, so its callers read the status here.  Synchronises with the last
 * extraction's stream; flags (nullable) receives `batch` ints, *any their OR. */
#define ORBX_STATUS_NODE_OVERFLOW 1
#define ORBX_STATUS_ITERATIONS 2
int orbx_extractor_status(orbx_extractor* ex, int batch, int* flags, int* any);
/* The same without synchronising: the device array of per-frame status words (int32
 * [last batch]), valid after the last extraction's stream reaches that point and until
 * the next extraction. */
int orbx_extractor_status_device(orbx_extractor* ex, const int32_t** d_status);
/* Test hook: cap every level's octree node capacity at `cap` (0 = the bound the
 * reference's algorithm guarantees, max(N+4, 4*nIni+4) per level), so that the overflow
 * status can be exercised.  Frees the extractor's buffers (pyramids included) after
 * draining the whole device; takes effect at the next extraction. */
int orbx_extractor_set_node_capacity(orbx_extractor* ex, int cap);

/* Level 0 of the pyramid is the input image (ORBextractor.cc:1688-1690).  With enable = 1,
 * orbx_extract_batch_device reads it in place from the caller's device frames instead of
 * copying it into the extractor's pyramid (when the frames are 16-byte aligned, their
 * frame pitch a multiple of 16 and their row stride a multiple of 64; otherwise it is
 * copied as before).  The frames must then stay unchanged while the pyramid is in use:
 * orbx_pyramid_level(_device) returns level 0 from them, and the stereo matchers
 * (orbx_compute_stereo_matches(_batch_device)) read the octave-0 SAD windows of
 * Frame::ComputeStereoMatches (Frame.cc:800-835) there.  Frames in a pitched layout
 * (rows a multiple of 64 bytes apart) qualify at any width. */
int orbx_extractor_set_level0_in_place(orbx_extractor* ex, int enable);

/* Per-stage HIP-event timing (ms) of extraction calls, averaged over the (up to 64)
 * most recent calls made since orbx_extractor_set_timing(ex, 1), which also resets the
 * average.  Events are recorded on the launch stream between the stages, so a timed
 * loop is measured without synchronising inside it.  Names are static strings.
 * enable = 2 + s (s = 0 pyramid .. 4 describe) records only stage s's two boundary events
 * (each recorded event costs the pipelined step ~0.2 %: bench.py times one stage live);
 * stage_times then returns that stage alone. */
int orbx_extractor_set_timing(orbx_extractor* ex, int enable);
int orbx_extractor_stage_times(orbx_extractor* ex, int max_stages, const char** names, float* ms,
                               int* n_stages);

/* mvImagePyramid[level] of frame `frame` of the last extraction: copies the level
 * ROI (w x h) into host memory `dst` with row stride dst_stride. */
int orbx_pyramid_level(orbx_extractor* ex, int frame, int level, uint8_t* dst, size_t dst_stride,
                       int* w, int* h);
/* Device pointer + row pitch of a pyramid level of the last device extraction. */
int orbx_pyramid_level_device(orbx_extractor* ex, int frame, int level, const uint8_t** d_ptr,
                              size_t* pitch, int* w, int* h);

/* ORBmatcher::DescriptorDistance on two 32-byte host descriptors; returns 0..256. */
int orbx_hamming(const uint8_t* a32, const uint8_t* b32);

/* dist[i*nb + j] = Hamming(a_i, b_j) for device descriptor arrays (32 B rows). */
int orbx_hamming_matrix_device(const uint8_t* d_a, int na, const uint8_t* d_b, int nb,
                               int32_t* d_dist, void* stream);

/* Windowed candidate scoring shared by the SearchByProjection overloads and
 * SearchForTriangulation: for query q (32 B descriptor at d_qdesc + 32*q) the
 * candidates are d_cand[d_cand_off[q] .. d_cand_off[q+1]) (indices into the target
 * descriptor array, in the reference's iteration order).  Outputs per query:
 * best/second-best distance, best candidate position (index into the target array,
 * -1 if none), and the target levels of best and second (as SearchByProjection
 * tracks them, ORBmatcher.cc:140-152).  `tie_last` = 0: strict < keeps the first
 * equal candidate (SearchByProjection); 1: the last equal candidate wins the best
 * slot (SearchForTriangulation, ORBmatcher.cc:955).  Device pointers, async. */
int orbx_window_match_device(const uint8_t* d_qdesc, int nq, const uint8_t* d_tdesc,
                             const int32_t* d_tlevel, const int32_t* d_cand_off,
                             const int32_t* d_cand, int tie_last, int32_t* d_best_idx,
                             int32_t* d_best_dist, int32_t* d_best_level, int32_t* d_second_dist,
                             int32_t* d_second_level, void* stream);

/* Host-pointer convenience wrapper of orbx_window_match_device (synchronous). */
int orbx_window_match(int device, const uint8_t* qdesc, int nq, const uint8_t* tdesc, int nt,
                      const int32_t* tlevel, const int32_t* cand_off, const int32_t* cand,
                      int tie_last, int32_t* best_idx, int32_t* best_dist, int32_t* best_level,
                      int32_t* second_dist, int32_t* second_level);

/* ------------------------------------------------------------------ matcher */

/* The Frame / KeyFrame fields the ORBmatcher functions read (include/Frame.h,
 * include/KeyFrame.h), as plain host arrays. */
typedef struct {
    int n;                       /* N */
    const orbx_keypoint* keys;   /* mvKeysUn */
    const uint8_t* desc;         /* mDescriptors, n x 32 */
    const float* u_right;        /* mvuRight (n) or NULL (monocular) */
    float fx, fy, cx, cy, bf, b; /* fx, fy, cx, cy, mbf, mb */
    float min_x, max_x, min_y, max_y; /* mnMinX, mnMaxX, mnMinY, mnMaxY */
    int nlevels;
    const float* scale_factors;  /* mvScaleFactors */
    const float* level_sigma2;   /* mvLevelSigma2 */
    float Tcw[12];               /* mTcw rows 0..2, row-major */
} orbx_frame_view;

/* MapPoint fields, indexed by MapPoint id (the ids stand in for MapPoint*).  Fields a
 * call does not read may be NULL: max/min_distance and normal are read only by the
 * KeyFrame / Sim3 projections (a13, a14).  n < 2^30 for the projection searches (their
 * claims carry a flag in bit 30; larger tables fail with ORBX_ERR_ARG). */
typedef struct {
    int n;
    const float* pos;            /* GetWorldPos(), n x 3 (may be NULL where unused) */
    const uint8_t* desc;         /* GetDescriptor(), n x 32 */
    const int32_t* observations; /* Observations() */
    const uint8_t* bad;          /* isBad() or NULL */
    const float* max_distance;   /* mfMaxDistance (GetMaxDistanceInvariance() = 1.2f * it) */
    const float* min_distance;   /* mfMinDistance (GetMinDistanceInvariance() = 0.8f * it) */
    const float* normal;         /* GetNormal(), n x 3 */
} orbx_mappoints;

/* Frame::IsInFrustum outputs per MapPoint id (Frame.cc:412-477), read by
 * SearchByProjection(Frame&, vector<MapPoint*>, th). */
typedef struct {
    const uint8_t* in_view;      /* mbTrackInView */
    const float* proj_x;         /* mTrackProjX */
    const float* proj_y;         /* mTrackProjY */
    const float* proj_xr;        /* mTrackProjXR */
    const int32_t* scale_level;  /* mnTrackScaleLevel */
    const float* view_cos;       /* mTrackViewCos */
} orbx_track;

typedef struct orbx_matcher orbx_matcher;

/* Failure of the sequential replay (every SearchByProjection form): its fixpoint has an
 * iteration guard that no valid input reaches.  The single-call forms below then return
 * ORBX_ERR_STATE (the MapPoint output is partial); the batched device forms
 * (orbx_match_sequence_device(_ex), orbx_search_local_points_device) write -1 into that
 * frame's nmatches entry, which a caller must treat as a failed frame, never as a count. */

/* ORBmatcher::ORBmatcher(nnratio, checkOri) (ORBmatcher.h:57), bound to HIP device
 * `device` with its own stream and scratch buffers. */
int orbx_matcher_create(int device, float nnratio, int check_ori, orbx_matcher** out);
void orbx_matcher_destroy(orbx_matcher* m);

/* SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, const float th)
 * ORBmatcher.cc:61-173.  frame_mp (F.mvpMapPoints as MapPoint ids, -1 = NULL) is
 * updated in place; queries = vpMapPoints ids in order. */
int orbx_search_by_projection_local(orbx_matcher* m, const orbx_frame_view* f, int32_t* frame_mp,
                                    const int32_t* queries, int nq, const orbx_mappoints* mps,
                                    const orbx_track* trk, float th, int* nmatches);

/* SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono)
 * ORBmatcher.cc:1620-1789 (TrackWithMotionModel, Tracking.cc:966-994). */
int orbx_search_by_projection_frame(orbx_matcher* m, const orbx_frame_view* cur, int32_t* cur_mp,
                                    const orbx_frame_view* last, const int32_t* last_mp,
                                    const uint8_t* last_outlier, const orbx_mappoints* mps, float th,
                                    int mono, int* nmatches);

/* SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound,
 * th, ORBdist) ORBmatcher.cc:1792-1924 (relocalisation, Tracking.cc:1629-1653).  kf: the
 * KeyFrame's keypoints (angles for the rotation check), kf_mp: GetMapPointMatches() as ids
 * (-1 = NULL), already_found: per MapPoint id (sAlreadyFound) or NULL.  cur_mp
 * (CurrentFrame.mvpMapPoints as ids) is updated in place.  Reads mps pos, desc, bad,
 * max_distance, min_distance. */
int orbx_search_by_projection_keyframe(orbx_matcher* m, const orbx_frame_view* cur, int32_t* cur_mp,
                                       const orbx_frame_view* kf, const int32_t* kf_mp,
                                       const uint8_t* already_found, const orbx_mappoints* mps, float th,
                                       int orb_dist, int* nmatches);

/* SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints,
 * vector<MapPoint*>& vpMatched, int th) ORBmatcher.cc:398-520 (LoopClosing::ComputeSim3,
 * LoopClosing.cc:417).  Scw: 3x4 row-major [sR | st].  points: vpPoints as ids; matched:
 * vpMatched as ids (kf->n entries, -1 = NULL), updated in place.  Reads mps pos, desc,
 * bad, max_distance, min_distance, normal. */
int orbx_search_by_projection_sim3(orbx_matcher* m, const orbx_frame_view* kf, const float* Scw,
                                   const int32_t* points, int npoints, int32_t* matched,
                                   const orbx_mappoints* mps, int th, int* nmatches);

/* Batched TrackWithMotionModel matching (Tracking.cc:966-994) over a device-resident
 * sequence produced by orbx_extract_batch_device: for b >= 1, frame b (CurrentFrame)
 * is matched against frame b-1 (LastFrame) with SearchByProjection(..., th, bMono=1)
 * semantics (ORBmatcher.cc:1620-1789).  Every keypoint i of frame b-1 carries
 * MapPoint id i at depth `depth` on its viewing ray (Observations() > 0).  d_Tcw: B x 12
 * floats (rows 0..2 of each mTcw).  Outputs (device): d_cur_mp [B][cap] (frame 0 stays
 * -1) and d_nmatches [B].  Asynchronous on `stream` (or the matcher's stream). */
int orbx_match_sequence_device(orbx_matcher* m, int batch, const orbx_keypoint* d_kps, const uint8_t* d_desc,
                               const int32_t* d_n, int cap, const float* d_Tcw, float fx, float fy, float cx,
                               float cy, float min_x, float max_x, float min_y, float max_y,
                               const float* scale_factors, int nlevels, float depth, float th,
                               int32_t* d_cur_mp, int32_t* d_nmatches, void* stream);

/* The general form: a sequence of Frames in the orbx_extract_batch_device layout, for
 * b >= 1 frame b (CurrentFrame) matched against frame b-1 (LastFrame) with
 * SearchByProjection(CurrentFrame, LastFrame, th, mono) (ORBmatcher.cc:1620-1789),
 * including the stereo / RGB-D octave ranges for motion along the optical axis
 * (bForward / bBackward, cc:1650-1701) and the mvuRight check (cc:1722-1729).
 * LastFrame keypoint i's MapPoint (id i, Observations() > 0) sits at mp_pos
 * (LastFrame.mvpMapPoints[i]->GetWorldPos()) or, without mp_pos, at `depth` on its
 * viewing ray; has_mp clears keypoints with no MapPoint or flagged mvbOutlier. */
typedef struct {
    int batch;                    /* B frames */
    const orbx_keypoint* kps;     /* [B][cap] mvKeysUn (device) */
    const uint8_t* desc;          /* [B][cap][32] mDescriptors */
    const int32_t* n;             /* [B] keypoint counts */
    int cap;
    const float* Tcw;             /* [B][12] mTcw rows 0..2 (device) */
    const float* u_right;         /* [B][cap] mvuRight (device) or NULL */
    const float* mp_pos;          /* [B][cap][3] (device) or NULL */
    const uint8_t* has_mp;        /* [B][cap] (device) or NULL = every keypoint */
    float depth;                  /* MapPoint depth when mp_pos is NULL */
    float fx, fy, cx, cy, bf, b;  /* fx, fy, cx, cy, mbf, mb (mb > 0 unless mono) */
    float min_x, max_x, min_y, max_y;
    int nlevels;
    const float* scale_factors;   /* host: mvScaleFactors (nlevels) */
    float th;
    int mono;                     /* bMono */
    int global_ids;               /* 0: MapPoint id = LastFrame keypoint index i; 1: id = (b-1)*cap + i */
    int32_t* cur_mp;              /* [B][cap] out: CurrentFrame.mvpMapPoints as MapPoint ids, -1 */
    int32_t* nmatches;            /* [B] out (frame 0: 0) */
    const int32_t* mp_obs;        /* [B*cap] Observations() per MapPoint id (device; needs global_ids), or
                                     NULL: every MapPoint has Observations() > 0.  A claim by a MapPoint
                                     with 0 observations (UpdateLastFrame's temporal points) does not
                                     block the keypoint (ORBmatcher.cc:1716-1718) */
    int retry_below;              /* TrackWithMotionModel's retry (Tracking.cc:988-994): a pair with fewer
                                     than retry_below matches is searched again from an empty
                                     mvpMapPoints at 2*th (the reference: 20); 0 = one search */
} orbx_sequence;
int orbx_match_sequence_device_ex(orbx_matcher* m, const orbx_sequence* seq, void* stream);

/* Tracking::SearchLocalPoints (Tracking.cc:1280-1336) for B Frames in HBM -- the
 * per-frame TrackLocalMap search.  For frame b:
 *   1. mvpMapPoints (frame_mp [b][cap], MapPoint ids, -1 = NULL; e.g. the
 *      orbx_match_sequence_device_ex output with global ids): bad MapPoints are set to
 *      NULL, the rest are "seen" and not projected again (Tracking.cc:1286-1299);
 *   2. Frame::IsInFrustum(pMP, viewing_cos_limit) (Frame.cc:412-477) for every entry of
 *      frame b's local map (mvpLocalMapPoints, local_ids[local_off[b] .. local_off[b+1]))
 *      that is neither seen nor bad;
 *   3. SearchByProjection(F, vpLocalMapPoints, th) (ORBmatcher.cc:61-173) with the
 *      matcher's nnratio (Tracking uses ORBmatcher(0.8)) over the points in view, in list
 *      order: frame_mp is updated in place, nmatches [b] receives its count.
 * MapPoints live in a device table indexed by id.  local_off is a host array (B + 1
 * ints: it sizes the launch); every other pointer is a device pointer.  cap must stay
 * below 8192 (keypoints); a local map may hold up to 2^20 MapPoints.  Asynchronous on
 * `stream` (or the matcher's). */
typedef struct {
    int n;                        /* MapPoints in the table */
    const float* pos;             /* [n][3] GetWorldPos() */
    const uint8_t* desc;          /* [n][32] GetDescriptor() */
    const float* normal;          /* [n][3] GetNormal() */
    const float* max_distance;    /* [n] mfMaxDistance */
    const float* min_distance;    /* [n] mfMinDistance */
    const int32_t* observations;  /* [n] Observations() */
    const uint8_t* bad;           /* [n] isBad() or NULL */
} orbx_mappoints_device;

typedef struct {
    int batch;
    const orbx_keypoint* kps;     /* [B][cap] mvKeysUn */
    const uint8_t* desc;          /* [B][cap][32] mDescriptors */
    const int32_t* n;             /* [B] keypoint counts */
    int cap;
    const float* u_right;         /* [B][cap] mvuRight or NULL */
    const float* Tcw;             /* [B][12] mTcw rows 0..2 */
    float fx, fy, cx, cy, bf;
    float min_x, max_x, min_y, max_y;
    int nlevels;
    const float* scale_factors;   /* host: mvScaleFactors (nlevels) */
    const int32_t* local_off;     /* host: [B + 1] */
    const int32_t* local_ids;     /* device: local map MapPoint ids, frame after frame; ids (here and in
                                     frame_mp) must be < mps->n: an id outside the table is treated as
                                     a NULL entry (never read out of bounds) */
    float th;                     /* 1; 3 for RGB-D; 5 right after a relocalisation (Tracking.cc:1320-1331) */
    float viewing_cos_limit;      /* 0.5 (Tracking.cc:1314) */
    int32_t* frame_mp;            /* [B][cap] in/out */
    int32_t* nmatches;            /* [B] out */
} orbx_local_map_batch;
int orbx_search_local_points_device(orbx_matcher* m, const orbx_mappoints_device* mps,
                                    const orbx_local_map_batch* lm, void* stream);

/* ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches)
 * (ORBmatcher.cc:228-392; Tracking::TrackReferenceKeyFrame / Relocalization).
 * kf_mp[i]: MapPoint id of KF keypoint i, -1 for NULL or isBad().  FeatureVectors as
 * CSR (nodes ascending, indices ascending within a node).  matches [f->n] out: the KF
 * MapPoint id matched to each frame keypoint, -1 = none.  Uses the matcher's nnratio
 * and checkOri. */
int orbx_search_by_bow_frame(orbx_matcher* m, const orbx_frame_view* kf, const int32_t* kf_mp,
                             const int32_t* kf_fv_node, const int32_t* kf_fv_off, const int32_t* kf_fv_idx,
                             int kf_fv_n, const orbx_frame_view* f, const int32_t* f_fv_node, const int32_t* f_fv_off,
                             const int32_t* f_fv_idx, int f_fv_n, int32_t* matches, int* nmatches);

/* ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
 * (ORBmatcher.cc:696-839; LoopClosing::ComputeSim3).  mp1 / mp2: MapPoint ids, -1 for
 * NULL or isBad().  matches12 [kf1->n] out: KF2's MapPoint id matched to each KF1
 * keypoint, -1 = none. */
int orbx_search_by_bow_keyframes(orbx_matcher* m, const orbx_frame_view* kf1, const int32_t* mp1,
                                 const int32_t* fv1_node, const int32_t* fv1_off, const int32_t* fv1_idx, int fv1_n,
                                 const orbx_frame_view* kf2, const int32_t* mp2, const int32_t* fv2_node,
                                 const int32_t* fv2_off, const int32_t* fv2_idx, int fv2_n, int32_t* matches12,
                                 int* nmatches);

/* ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
 * vector<int>& vnMatches12, int windowSize) (ORBmatcher.cc:539-683;
 * Tracking::MonocularInitialization).  prev_matched [f1->n][2] in/out; matches12
 * [f1->n] out (F2 index or -1).  Frames of up to 2^20 keypoints whose working set
 * fits one workgroup's LDS (16 B per keypoint: n1, n2 <= ~8k). */
int orbx_search_for_initialization(orbx_matcher* m, const orbx_frame_view* f1, const orbx_frame_view* f2,
                                   float* prev_matched, int32_t* matches12, int window_size, int* nmatches);

/* ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, float th)
 * (ORBmatcher.cc:1067-1221; LocalMapping::SearchInNeighbors): the search part.  For
 * each points[k] (MapPoint id, -1 = NULL) not flagged in skip[id] (isBad() ||
 * IsInKeyFrame(pKF)), best[k] receives the KF keypoint it fuses with (distance <=
 * TH_LOW, Fuse's chi-square gate on mvuRight) or -1.  No MapPoint's search depends on
 * another's, so all run at once; the caller then runs the reference's Replace /
 * AddObservation loop in order over best[], re-checking isBad() / IsInKeyFrame(). */
int orbx_fuse(orbx_matcher* m, const orbx_frame_view* kf, const int32_t* points, int npoints, const uint8_t* skip,
              const orbx_mappoints* mps, float th, int32_t* best);

/* ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, float th,
 * vector<MapPoint*>& vpReplacePoint) (ORBmatcher.cc:1226-1352; LoopClosing::SearchAndFuse):
 * the search part; skip[id] = isBad() || pKF->GetMapPoints().count(pMP).  Scw: 3 x 4
 * row-major [sR | st]. */
int orbx_fuse_sim3(orbx_matcher* m, const orbx_frame_view* kf, const float* Scw, const int32_t* points, int npoints,
                   const uint8_t* skip, const orbx_mappoints* mps, float th, int32_t* best);

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
 * (ORBmatcher.cc:1361-1602; LoopClosing::ComputeSim3).  mp1 / mp2: GetMapPointMatches()
 * as ids (-1 = NULL); already1 / already2: vbAlreadyMatched1/2 from the incoming
 * vpMatches12 (may be NULL = none); R12 row-major 3 x 3, t12 3.  matches12 [kf1->n]
 * in/out (KF2 MapPoint ids): mutual matches are written, other entries are left as
 * they are.  *nfound = number written. */
int orbx_search_by_sim3(orbx_matcher* m, const orbx_frame_view* kf1, const int32_t* mp1, const uint8_t* already1,
                        const orbx_frame_view* kf2, const int32_t* mp2, const uint8_t* already2,
                        const orbx_mappoints* mps, float s12, const float* R12, const float* t12, float th,
                        int32_t* matches12, int* nfound);

/* MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:295-360) for nmp MapPoints at once:
 * MapPoint k's descriptors (good observations, observation-map order) are
 * desc[off[k] .. off[k+1]) (32 B each).  best[k] = index within that list of the
 * descriptor with the smallest median distance (-1 when empty); out_desc [nmp][32]
 * (optional) receives it. */
int orbx_compute_distinctive_descriptors(int device, int nmp, const int32_t* off, const uint8_t* desc, int32_t* best,
                                         uint8_t* out_desc);
int orbx_compute_distinctive_descriptors_device(int nmp, const int32_t* d_off, const uint8_t* d_desc, int32_t* d_best,
                                                uint8_t* d_out_desc, void* stream);

/* Footprint of orbx_match_sequence_device's search: 0 (default) = one 1024-thread
 * workgroup per problem with keypoint descriptors and query state in LDS (fastest alone);
 * 1 = 256 threads and global-memory query state; 2 = split into three launches (grid
 * sort per problem, scoring spread over all problems' queries, one wave per problem for
 * the ordered commit); 3 = one wave per problem; 4 = lean: 1024 threads with only the
 * sorted grid and the claims in LDS (descriptors, query state and angles in global
 * memory), the form that leaves the most LDS to extraction running concurrently on
 * another stream; 5 = lean split: mode 4's workgroup sorts and scores, then a one-wave
 * kernel with only the claims in LDS replays.  Same results in every mode. */
int orbx_matcher_set_footprint(orbx_matcher* m, int mode);

/* HIP-event timing of orbx_match_sequence_device and orbx_compute_stereo_matches_batch_device:
 * milliseconds averaged over the (up to 64) most recent calls since
 * orbx_matcher_set_timing(m, 1). */
int orbx_matcher_set_timing(orbx_matcher* m, int enable);
int orbx_matcher_last_ms(orbx_matcher* m, float* ms);
/* Wall time (microseconds) of the newest drop-in host call on m (the SearchByProjection
 * overloads, SearchForTriangulation, SearchByBoW, SearchForInitialization, Fuse,
 * SearchBySim3, ComputeStereoMatches): entry to return, i.e. what a C++ caller such as
 * Tracking pays per call, without any binding overhead.  -1 for a null matcher. */
double orbx_matcher_last_call_us(const orbx_matcher* m);

/* SearchForTriangulation(KF1, KF2, F12, vMatchedPairs, bOnlyStereo)
 * ORBmatcher.cc:850-1056 (LocalMapping::CreateNewMapPoints, LocalMapping.cc:305).
 * DBoW2 FeatureVectors as CSR: node ids ascending (fv_node[k]), keypoints of node k
 * at fv_idx[fv_off[k] .. fv_off[k+1]).  pairs receives (idx1, idx2) in idx1 order
 * (capacity 2*kf1->n ints); *npairs the count. */
int orbx_search_for_triangulation(orbx_matcher* m, const orbx_frame_view* kf1, const uint8_t* kf1_has_mp,
                                  const int32_t* fv1_node, const int32_t* fv1_off, const int32_t* fv1_idx,
                                  int fv1_n, const orbx_frame_view* kf2, const uint8_t* kf2_has_mp,
                                  const int32_t* fv2_node, const int32_t* fv2_off, const int32_t* fv2_idx,
                                  int fv2_n, const float* F12, int only_stereo, int32_t* pairs, int* npairs);

/* One KeyFrame as SearchForTriangulation reads it, left in HBM by the batched device
 * calls (frame b of their [B][cap] layouts): orbx_extract_batch_device (keys, desc, n),
 * orbx_compute_stereo_matches_batch_device (u_right), orbx_vocabulary_transform_batch_device
 * (the FeatureVector CSR fv_node / fv_off / fv_idx / nfv).  Device pointers, except Tcw:
 * the pose stays a host value as in the reference (KeyFrame::GetPose). */
typedef struct {
    const orbx_keypoint* keys;   /* mvKeysUn (cap slots) */
    const uint8_t* desc;         /* mDescriptors (cap x 32) */
    const int32_t* n;            /* N (one device int; min(*n, cap) keypoints are read) */
    const float* u_right;        /* mvuRight (cap) or NULL (monocular) */
    const uint8_t* has_mp;       /* GetMapPoint(i) != NULL (cap) */
    const int32_t* fv_node;      /* mFeatVec node ids, ascending (cap) */
    const int32_t* fv_off;       /* node k's keypoints: fv_idx[fv_off[k] .. fv_off[k+1]) (cap + 1) */
    const int32_t* fv_idx;       /* (cap) */
    const int32_t* nfv;          /* node count (one device int) */
    float Tcw[12];               /* host: mTcw rows 0..2 */
} orbx_keyframe_device;

/* LocalMapping::CreateNewMapPoints' matching loop (LocalMapping.cc:235-305) over many
 * keyframe pairs at once: for p < npairs, SearchForTriangulation(KF1 = kfs[pairs[2p]],
 * KF2 = kfs[pairs[2p+1]], F12 + 9p, vMatchedPairs, only_stereo) (ORBmatcher.cc:850-1056),
 * with the matcher's checkOri (LocalMapping uses ORBmatcher(0.6, false)).  `cam` gives
 * the shared intrinsics fx, fy, cx, cy and the level tables (nlevels, scale_factors,
 * level_sigma2); its keys / desc / u_right / Tcw are not read.  pairs and F12 (row-major
 * 3x3, LocalMapping::ComputeF12) are host arrays; the epipole comes from the host poses.
 * Outputs (device): d_matches12 [P][cap] (vMatches12: KF2 index or -1), d_pairs
 * [P][cap][2] (vMatchedPairs, idx1 order) and d_npairs [P].  Enqueued on `stream` (or the
 * matcher's) without synchronising; the host tables are staged through pinned memory, so
 * they may be reused on return.  Successive calls on one matcher must use one stream
 * (they share its device work area).  cap <= 8192. */
int orbx_search_for_triangulation_batch_device(orbx_matcher* m, int nkf, const orbx_keyframe_device* kfs,
                                               const orbx_frame_view* cam, int npairs, const int32_t* pairs,
                                               const float* F12, int only_stereo, int cap, int32_t* d_matches12,
                                               int32_t* d_pairs, int32_t* d_npairs, void* stream);

/* Frame::ComputeStereoMatches (Frame.cc:673-885) of one stereo Frame, as the stereo Frame
 * constructor runs it (Frame.cc:99-178): the left image was extracted by `ex_left` (frame
 * `left_frame` of its last extraction, mpORBextractorLeft) and the right image by
 * `ex_right` (frame `right_frame`, mpORBextractorRight); the two may be one extractor
 * holding both images.  The SAD refinement reads both extractors' mvImagePyramid
 * (Frame.cc:782-818).  left: mvKeys / mDescriptors / mbf; keys_r / desc_r: mvKeysRight /
 * mDescriptorsRight.  maxD = mbf / minZ (this fork reads mb before it is set,
 * Frame.cc:711-713; upstream's value is fx).  Writes mvuRight and mvDepth (n_left floats
 * each, -1 = no match), including this fork's in-loop outlier pass (Frame.cc:868-884).
 * Host buffers; synchronous. */
int orbx_compute_stereo_matches(orbx_matcher* m, orbx_extractor* ex_left, int left_frame, orbx_extractor* ex_right,
                                int right_frame, const orbx_frame_view* left, const orbx_keypoint* keys_r,
                                const uint8_t* desc_r, int n_right, float max_disparity, float* u_right,
                                float* depth);

/* The same for B stereo Frames in HBM (configs[2]): pair b's left image is frame
 * left_frame0 + b of ex_left's last extraction with keypoints d_kps_l + b*cap
 * (min(d_n_l[b], cap) of them, the orbx_extract_batch_device layout), its right image
 * frame right_frame0 + b of ex_right's.  Scale factors come from the extractors.
 * Outputs d_u_right / d_depth [B][cap] (slots past a pair's count are -1).  Enqueued on
 * `stream` (or the matcher's) without synchronising: the caller orders it after both
 * extractions (and before either extractor's next extraction, which overwrites the
 * pyramids).  cap <= 8192. */
int orbx_compute_stereo_matches_batch_device(orbx_matcher* m, orbx_extractor* ex_left, int left_frame0,
                                             orbx_extractor* ex_right, int right_frame0, int batch,
                                             const orbx_keypoint* d_kps_l, const uint8_t* d_desc_l,
                                             const int32_t* d_n_l, const orbx_keypoint* d_kps_r,
                                             const uint8_t* d_desc_r, const int32_t* d_n_r, int cap, float bf,
                                             float max_disparity, float* d_u_right, float* d_depth, void* stream);

/* ---- Frame: undistortion and grid (§8(f) rank 3) ----
 * Camera intrinsics and distortion: Frame::mK and Frame::mDistCoef [k1 k2 p1 p2 (k3)]
 * (Tracking.cc:60-92; k3 = 0 when the settings have four coefficients). */
typedef struct {
    float fx, fy, cx, cy;
    float k1, k2, p1, p2, k3;
} orbx_camera;

/* Frame::UndistortKeyPoints (Frame.cc:586-628): cv::undistortPoints(mvKeys, K, D,
 * noArray(), K) on every keypoint; mvKeysUn = mvKeys when k1 == 0.  Host buffers of n
 * keypoints (keys_un may equal keys). */
int orbx_undistort_keypoints(int device, const orbx_camera* cam, const orbx_keypoint* keys, int n,
                             orbx_keypoint* keys_un);
/* Same over the orbx_extract_batch_device layout (frame b at d_keys + b*cap, min(d_n[b], cap)
 * keypoints) into d_keys_un [B][cap].  Asynchronous on `stream`. */
int orbx_undistort_keypoints_device(const orbx_camera* cam, int batch, const orbx_keypoint* d_keys,
                                    const int32_t* d_n, int cap, orbx_keypoint* d_keys_un, void* stream);
/* Frame::ComputeImageBounds (Frame.cc:636-665): bounds = {mnMinX, mnMaxX, mnMinY, mnMaxY}. */
int orbx_compute_image_bounds(int device, const orbx_camera* cam, int cols, int rows, float* bounds);
/* Frame::AssignFeaturesToGrid (Frame.cc:351-370, PosInGrid 558-567) as CSR: cell
 * c = ix * FRAME_GRID_ROWS + iy (64 x 48) holds cell_idx[cell_start[c] .. cell_start[c+1]),
 * ascending; keypoints outside the grid are left out.  n <= 8192. */
int orbx_assign_features_to_grid(int device, const orbx_keypoint* keys_un, int n, const float* bounds,
                                 int32_t* cell_start, int32_t* cell_idx);
/* Batched: d_cell_start [B][3073], d_cell_idx [B][cap], cap <= 8192.  Asynchronous. */
int orbx_assign_features_to_grid_device(int batch, const orbx_keypoint* d_keys_un, const int32_t* d_n, int cap,
                                        const float* bounds, int32_t* d_cell_start, int32_t* d_cell_idx,
                                        void* stream);

/* The MapPoints a stereo / RGB-D keyframe is born with (Tracking::CreateNewKeyFrame,
 * Tracking.cc:1069-1121) for B frames in HBM, as an orbx_mappoints_device table with id
 * b*cap + i: for every keypoint i < n[b] with depth z > 0 (d_depth [B][cap] = mvDepth, the
 * caller's selection of close points; or `const_depth` for every keypoint when d_depth is
 * NULL), pos = Frame::UnprojectStereo(i) (Frame.cc:912-927) and normal / mfMaxDistance /
 * mfMinDistance from MapPoint::UpdateNormalAndDepth with the frame as the only observation
 * (MapPoint.cc:386-439); observations 1, bad 0.  Other slots: bad 1, observations 0.
 * Outputs [B*cap] (pos, normal: x3).  scale_factors is a host array.  Asynchronous. */
int orbx_create_mappoints_device(int batch, const orbx_keypoint* d_kps, const int32_t* d_n, int cap,
                                 const float* d_depth, float const_depth, const float* d_Tcw, float fx, float fy,
                                 float cx, float cy, const float* scale_factors, int nlevels, float* d_pos,
                                 float* d_normal, float* d_max_distance, float* d_min_distance,
                                 int32_t* d_observations, uint8_t* d_bad, void* stream);

/* Tracking::UpdateLastFrame (Tracking.cc:893-954) for B stereo / RGB-D LastFrames in HBM
 * (none of them the last keyframe): the keypoints with mvDepth > 0 are visited nearest
 * first (pairs (depth, index) ascending); one without a MapPoint, or whose MapPoint has
 * Observations() < 1, gets a temporal MapPoint at Frame::UnprojectStereo(i) (Frame.cc:
 * 912-927) with Observations() 0; the walk ends after the first point beyond th_depth
 * (mThDepth = mbf * ThDepth / fx) once more than 100 points were visited.  In: d_obs_in
 * [B][cap] Observations() of LastFrame.mvpMapPoints (-1 = NULL) and d_pos_in [B][cap][3]
 * their world positions, or both NULL (no MapPoints).  Out: d_mp_obs [B][cap] (-1 = none),
 * d_mp_pos [B][cap][3], d_has_mp [B][cap] -- the orbx_sequence mp_obs / mp_pos / has_mp
 * inputs of the following TrackWithMotionModel search (global ids b*cap + i).  The outputs
 * may alias the inputs.  Asynchronous. */
int orbx_update_last_frame_device(int batch, const orbx_keypoint* d_kps, const int32_t* d_n, int cap,
                                  const float* d_depth, const float* d_Tcw, float fx, float fy, float cx, float cy,
                                  float th_depth, const int32_t* d_obs_in, const float* d_pos_in, int32_t* d_mp_obs,
                                  float* d_mp_pos, uint8_t* d_has_mp, void* stream);

/* ---- RGB-D Frame (configs[4]) ----
 * Frame::Frame(imGray, imDepth, ...) for RGB-D (Frame.cc:192-264) after ExtractORB:
 * UndistortKeyPoints (Frame.cc:586-628) and ComputeStereoFromRGBD (Frame.cc:888-909), with
 * Tracking::GrabImageRGBD's depth conversion (Tracking.cc:265-271) applied to the pixels the
 * lookup reads.  For keypoint i (mvKeys[i] = kps, mvKeysUn[i] = kps_un):
 *   d = imDepth.at<float>((int)kp.y, (int)kp.x), imDepth = the depth image converted to
 *       CV_32F with scale mDepthMapFactor (= 1 / DepthMapFactor, Tracking.cc:166-170):
 *       a u16 image always (d = (float)raw * factor), an f32 image only when
 *       |factor - 1| > 1e-5 (d = raw * factor), else as is;
 *   d > 0: mvDepth[i] = d, mvuRight[i] = kpU.x - mbf / d; otherwise both -1.
 * A keypoint outside the depth image (never one the extractor produced) gets -1 (the
 * reference's Mat::at would read out of bounds). */
#define ORBX_DEPTH_U16 0
#define ORBX_DEPTH_F32 1
typedef struct {
    int batch;                   /* B frames in the orbx_extract_batch_device layout */
    const orbx_keypoint* kps;    /* [B][cap] mvKeys (device): the depth lookup positions */
    orbx_keypoint* kps_un;       /* [B][cap] mvKeysUn (device): written when a camera is given,
                                    read otherwise */
    const int32_t* n;            /* [B] keypoint counts */
    int cap;
    const void* depth;           /* frame b's depth image at depth + b*frame_bytes, rows
                                    row_bytes apart (device) */
    int depth_type;              /* ORBX_DEPTH_U16 (TUM's 16-bit PNG) or ORBX_DEPTH_F32 */
    int width, height;           /* depth image size (the gray image's) */
    long long row_bytes, frame_bytes;
    float depth_map_factor;      /* Tracking's mDepthMapFactor (1 / DepthMapFactor) */
    float bf;                    /* mbf */
    float* u_right;              /* [B][cap] out: mvuRight (slots >= n[b]: -1) */
    float* depth_out;            /* [B][cap] out: mvDepth (slots >= n[b]: -1) */
} orbx_rgbd_batch;
/* cam non-NULL: UndistortKeyPoints into kps_un and the depth lookup in one pass; NULL:
 * kps_un holds mvKeysUn already.  Asynchronous on `stream`. */
int orbx_compute_stereo_from_rgbd_device(const orbx_camera* cam, const orbx_rgbd_batch* rb, void* stream);
/* One RGB-D Frame from host buffers (the drop-in Frame constructor): n keypoints, a
 * width x height depth image with rows row_bytes apart.  keys_un: out when cam is
 * non-NULL, else in.  u_right / depth_out: n floats. */
int orbx_compute_stereo_from_rgbd(int device, const orbx_camera* cam, const orbx_keypoint* keys, int n,
                                  const void* depth, int depth_type, int width, int height, size_t row_bytes,
                                  float depth_map_factor, float bf, orbx_keypoint* keys_un, float* u_right,
                                  float* depth_out);

/* ---- DBoW2 vocabulary (TemplatedVocabulary<FORB::TDescriptor, FORB>, §8(f) rank 1) ----
 * The tree lives in HBM as its CSR edge list.  Scoring / weighting
 * codes are DBoW2's enums (BowVector.h:29-56): scoring L1_NORM 0, L2_NORM 1,
 * CHI_SQUARE 2, KL 3, BHATTACHARYYA 4, DOT_PRODUCT 5; weighting TF_IDF 0, TF 1, IDF 2,
 * BINARY 3. */
typedef struct orbx_vocabulary orbx_vocabulary;

/* TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424; called by
 * System.cc:67): header "k L scoring weighting", then one node per line "parent
 * isLeaf d0..d31 weight".  Same header range checks; empty lines are skipped (the
 * reference turns a trailing one into a root child with an uninitialised descriptor);
 * a malformed node line or a parent id that does not precede the node is ORBX_ERR_ARG. */
int orbx_vocabulary_load_text_file(const char* path, int device, orbx_vocabulary** out);
/* Same from an in-memory text of `len` bytes. */
int orbx_vocabulary_load_text(const char* text, size_t len, int device, orbx_vocabulary** out);
void orbx_vocabulary_destroy(orbx_vocabulary* voc);
/* m_k, m_L, m_scoring, m_weighting, node count (incl. root), size() (words). */
int orbx_vocabulary_info(const orbx_vocabulary* voc, int* k, int* L, int* scoring, int* weighting, int* nnodes,
                         int* nwords);
/* The vocabulary's hipStream_t (as void*). */
void* orbx_vocabulary_stream(orbx_vocabulary* voc);

/* TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup)
 * (TemplatedVocabulary.h:1220-1259) for n descriptors (host buffers, n x 32 B).
 * node may be NULL.  A leaf reached above level L - levelsup reports the deepest
 * node (the reference leaves nid unset there). */
int orbx_vocabulary_transform_features(orbx_vocabulary* voc, const uint8_t* desc, int n, int levelsup,
                                       int32_t* word, double* weight, int32_t* node);

/* TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup)
 * (TemplatedVocabulary.h:1127-1186) for one frame of n <= 8192 descriptors (host
 * buffers), as called by Frame::ComputeBoW / KeyFrame::ComputeBoW with levelsup 4
 * (Frame.cc:573-583, KeyFrame.cc:66-74).  BowVector: (bow_word[j], bow_value[j]),
 * j < *nbow, ascending words.  FeatureVector: node fv_node[j] (ascending) holds the
 * features fv_idx[fv_off[j] .. fv_off[j+1]) (ascending), j < *nfv.  Capacities: n
 * entries, fv_off n + 1. */
int orbx_vocabulary_transform(orbx_vocabulary* voc, const uint8_t* desc, int n, int levelsup, int32_t* bow_word,
                              double* bow_value, int* nbow, int32_t* fv_node, int32_t* fv_off, int32_t* fv_idx,
                              int* nfv);

/* Batched device path over the orbx_extract_batch_device layout: frame b's
 * descriptors at d_desc + b*cap*32, min(d_n[b], cap) of them, cap <= 8192.  Outputs
 * (device) per frame: d_bow_word / d_bow_value / d_fv_node / d_fv_idx [B][cap],
 * d_fv_off [B][cap+1], d_nbow / d_nfv [B]; optional d_feat_word / d_feat_node [B][cap]
 * (the word and level-(L - levelsup) node of every feature; NULL = not wanted).
 * Asynchronous on `stream` (or the vocabulary's stream). */
int orbx_vocabulary_transform_batch_device(orbx_vocabulary* voc, int batch, const uint8_t* d_desc,
                                           const int32_t* d_n, int cap, int levelsup, int32_t* d_feat_word,
                                           int32_t* d_feat_node, int32_t* d_bow_word, double* d_bow_value,
                                           int32_t* d_nbow, int32_t* d_fv_node, int32_t* d_fv_off,
                                           int32_t* d_fv_idx, int32_t* d_nfv, void* stream);

/* HIP-event timing of transform calls (events on the launch stream), averaged over
 * the (up to 64) most recent calls: the tree walk and the per-frame vector build. */
int orbx_vocabulary_set_timing(orbx_vocabulary* voc, int enable);
int orbx_vocabulary_stage_times(orbx_vocabulary* voc, float* walk_ms, float* frame_ms);

/* Alternative kernel forms and diagnostics switches, process-wide (tests and A/B tools;
 * the product reads no environment).  Names: "pz_seg" (pyramid levels per launch, 0 = one
 * launch), "pz_byte" (byte-read k_pyramid), "desc_tiles" (tile-major describe),
 * "extract_dma" (single host call through DMA copies), "replay_threads" (64..1024),
 * "dup_stage" (launch extraction stage k twice), "oct_stamps" / "call_stamps" /
 * "match_stamps" (phase stamps to stderr).  value < 0 restores the default; name NULL
 * restores every default.  Every form gives the same results.  A frame size's plan reads
 * pz_seg / pz_byte / desc_tiles when an extractor first plans it. */
int orbx_debug_set(const char* name, int value);

/* Library / device info. */
const char* orbx_version(void);
int orbx_device_count(int* n);
const char* orbx_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_H */
