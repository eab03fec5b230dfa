/*
 * orbx_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Plain-C CPU restatement of ORB-SLAM2's per-frame ORB extraction and Hamming
 * matching hot path (reference: /root/reference, xcmworkharder/OrbSlam2CommentedByXcm).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The shipped HIP path (liborbx.so) never links or calls it.
 *
 * Parity status: "parity unpinned" against the reference binary.  The reference
 * path needs OpenCV 3.3.1 (Thirdparty/DBoW2/build/CMakeCache.txt:178), which is not
 * in this image, so the reference cannot be built here (writing header/library
 * stand-ins is not allowed), and the reference ships no tests or golden vectors.
 * The restatement is pinned by known-answer tests derived from the reference
 * source text (level sizes, per-level budgets, umax, pattern, fastAtan2 algebra,
 * FAST score algebra) and by a second, independent numpy restatement of the
 * pixel stages (tests/reference_numpy.py).  The OpenCV 3.3.1 internals it fixes
 * (resize, GaussianBlur, FAST, fastAtan2, cvRound) are documented in DESIGN.md.
 */
#ifndef ORBX_ORACLE_H
#define ORBX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORA_MAX_LEVELS 32

/* == cv::KeyPoint (pt.x, pt.y, size, angle, response, octave, class_id): 28 bytes */
typedef struct {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} ora_keypoint;

/* ORBextractor members (ORBextractor.h:204-219) computed as ORBextractor.cc:438-550 */
typedef struct {
    int nfeatures, nlevels, ini_th_fast, min_th_fast;
    double scale_factor; /* stored as double: ORBextractor.h:207 */
    float scale[ORA_MAX_LEVELS], inv_scale[ORA_MAX_LEVELS];
    float sigma2[ORA_MAX_LEVELS], inv_sigma2[ORA_MAX_LEVELS];
    int features_per_level[ORA_MAX_LEVELS];
    int umax[16];
} ora_params;

int ora_params_init(ora_params* p, int nfeatures, float scale_factor, int nlevels,
                    int ini_th_fast, int min_th_fast);
void ora_level_size(const ora_params* p, int W, int H, int level, int* w, int* h);

/* OpenCV 3.3.1 primitives as used on the path (semantics fixed in DESIGN.md §OpenCV) */
int ora_cv_round(double v);
int ora_cv_roundf(float v);
float ora_fast_atan2(float y, float x);
void ora_resize_linear_u8(const uint8_t* src, int sw, int sh, size_t sstride,
                          uint8_t* dst, int dw, int dh, size_t dstride);
void ora_gaussian_blur7_u8(const uint8_t* src, int w, int h, size_t sstride,
                           uint8_t* dst, size_t dstride);
int ora_fast_corner_score(const uint8_t* p, int stride, int threshold);
int ora_fast_detect(const uint8_t* img, int rows, int cols, size_t stride, int threshold,
                    ora_keypoint* out, int cap);

/* ORB-SLAM2 stages */
float ora_ic_angle(const uint8_t* img, size_t stride, float x, float y, const int* umax);
void ora_cos_sin(float angle_deg, float* c, float* s);
/* 0: (float)cos((double)r) (default); 1: cosf / sinf as ORBextractor.cc:123-125 (calling thread) */
void ora_set_trig_mode(int mode);
void ora_set_contract_mode(int mode); /* H4: 1 fused rBRIEF sample offsets (shipped), 0 unfused */
void ora_set_octree_tie_mode(int mode);
long ora_octree_ties(int reset);
void ora_orb_descriptor(const uint8_t* img, size_t stride, float x, float y, float angle_deg,
                        uint8_t* desc);
int ora_distribute_octree(const ora_keypoint* keys, int n, int minX, int maxX, int minY,
                          int maxY, int N, ora_keypoint* out, int cap);

/* Pyramid: levels[l] receives w_l*h_l bytes (row stride w_l). */
int ora_pyramid(const ora_params* p, const uint8_t* img, int W, int H, size_t stride,
                uint8_t** levels);

/* Per-level FAST candidates (vToDistributeKeys, coordinates relative to minBorder). */
int ora_level_candidates(const ora_params* p, const uint8_t* level, int w, int h, ora_keypoint* out,
                         int cap);
int ora_level_candidates_cells(const ora_params* p, const uint8_t* level, int w, int h, ora_keypoint* out,
                               int cap, int* cell_counts, int cell_cap, int* ncells);

/* Full ORBextractor::operator() (ORBextractor.cc:1513-1629).  Returns the keypoint
 * count (>=0), or -1 if cap is too small.  level_counts (nullable) receives the
 * per-level kept counts. */
int ora_extract(const ora_params* p, const uint8_t* img, int W, int H, size_t stride,
                ora_keypoint* kps, uint8_t* desc, int cap, int* level_counts);

/* ORBmatcher::DescriptorDistance (ORBmatcher.cc:1983-2003) */
int ora_descriptor_distance(const uint8_t* a, const uint8_t* b);

#ifdef __cplusplus
}
#endif
#endif
