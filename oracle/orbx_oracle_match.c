/*
 * orbx_oracle_match.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the ORBmatcher /
 * Frame matching functions on the hot path (parity checker, never the product).
 *
 *   AssignFeaturesToGrid / PosInGrid / GetFeaturesInArea   Frame.cc:351-370, 488-567
 *   ComputeThreeMaxima                                      ORBmatcher.cc:1935-1977
 *   SearchByProjection(Frame&, vector<MapPoint*>, th)       ORBmatcher.cc:61-173 (a11)
 *   SearchByProjection(Frame&, const Frame&, th, bMono)     ORBmatcher.cc:1620-1789 (a12)
 *   SearchForTriangulation(KF1, KF2, F12, pairs, stereo)    ORBmatcher.cc:850-1056 (a15)
 *   Frame::ComputeStereoMatches                             Frame.cc:673-885 (a18)
 *
 * Object-graph inputs (Frame, MapPoint, KeyFrame, FeatureVector) are passed as the
 * plain arrays they hold.  Geometric products (Rcw*x + t) are evaluated in float,
 * left to right -- OpenCV 3.3.1's small-matrix gemm accumulation is not pinned here
 * ("parity unpinned").
 */
#include "orbx_oracle_match.h"

#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

enum { TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30 };

/* ---------------------------------------------------------------- grid */

/* Frame::PosInGrid, Frame.cc:558-567 */
/* Hazard H4 in the matchers.  g++ -O3 -march=native (the reference's flags) contracts
 * the projection and epipolar expressions -- GCC fuses the first product of a sum into an
 * FMA -- and so does this restatement (and liborbx): u =
 * fma(fx*xc, invzc, cx), ur = fma(-mbf, invzc, u), CheckDistEpipolarLine's
 * fma(x, F00, y*F10) + F20, fma(a, x2, b*y2) + c, fma(a, a, b*b), the epipole test's
 * fma(dx, dx, dy*dy), Fuse's chi-square fma(er, er, fma(ex, ex, ey*ey)).
 * ora_set_match_contract_mode(0) switches the process to the unfused forms so the effect
 * can be counted (tests/h4_match_contract_count.py). */
static int g_mcontract = 1;  /* process-wide: cleared only by the exposure script */
void ora_set_match_contract_mode(int mode) { g_mcontract = mode; }
/* a*b + c */
static inline float mad_(float a, float b, float c) { return g_mcontract ? fmaf(a, b, c) : a * b + c; }
/* c - a*b */
static inline float msub_(float c, float a, float b) { return g_mcontract ? fmaf(-a, b, c) : c - a * b; }

static int pos_in_grid(const ora_frame* f, float inv_w, float inv_h, const ora_keypoint* kp, int* px, int* py) {
    *px = (int)roundf((kp->x - f->min_x) * inv_w);
    *py = (int)roundf((kp->y - f->min_y) * inv_h);
    if (*px < 0 || *px >= ORA_GRID_COLS || *py < 0 || *py >= ORA_GRID_ROWS) return 0;
    return 1;
}

/* Frame::AssignFeaturesToGrid, Frame.cc:351-370 (grid cell lists in index order);
 * mfGridElementWidthInv = FRAME_GRID_COLS / (mnMaxX - mnMinX), Frame.cc:157-159 */
void ora_grid_build(const ora_frame* f, ora_grid* g) {
    g->inv_w = (float)ORA_GRID_COLS / (f->max_x - f->min_x);
    g->inv_h = (float)ORA_GRID_ROWS / (f->max_y - f->min_y);
    int* cnt = (int*)calloc(ORA_GRID_COLS * ORA_GRID_ROWS, sizeof(int));
    int* cell = (int*)malloc(sizeof(int) * (size_t)(f->n ? f->n : 1));
    for (int i = 0; i < f->n; i++) {
        int px, py;
        if (pos_in_grid(f, g->inv_w, g->inv_h, &f->keys[i], &px, &py)) {
            cell[i] = px * ORA_GRID_ROWS + py;
            cnt[cell[i]]++;
        } else
            cell[i] = -1;
    }
    g->start[0] = 0;
    for (int c = 0; c < ORA_GRID_COLS * ORA_GRID_ROWS; c++) g->start[c + 1] = g->start[c] + cnt[c];
    g->idx = (int*)malloc(sizeof(int) * (size_t)(g->start[ORA_GRID_COLS * ORA_GRID_ROWS] + 1));
    memset(cnt, 0, sizeof(int) * ORA_GRID_COLS * ORA_GRID_ROWS);
    for (int i = 0; i < f->n; i++)
        if (cell[i] >= 0) g->idx[g->start[cell[i]] + cnt[cell[i]]++] = i;
    free(cnt);
    free(cell);
}

void ora_grid_free(ora_grid* g) {
    free(g->idx);
    g->idx = NULL;
}

/* Frame::GetFeaturesInArea, Frame.cc:488-548 */
int ora_features_in_area(const ora_frame* f, const ora_grid* g, float x, float y, float r, int minLevel,
                         int maxLevel, int* out, int cap) {
    int n = 0;
    int t;
    t = (int)floorf((x - f->min_x - r) * g->inv_w);
    const int nMinCellX = t > 0 ? t : 0;
    if (nMinCellX >= ORA_GRID_COLS) return 0;
    t = (int)ceilf((x - f->min_x + r) * g->inv_w);
    const int nMaxCellX = t < ORA_GRID_COLS - 1 ? t : ORA_GRID_COLS - 1;
    if (nMaxCellX < 0) return 0;
    t = (int)floorf((y - f->min_y - r) * g->inv_h);
    const int nMinCellY = t > 0 ? t : 0;
    if (nMinCellY >= ORA_GRID_ROWS) return 0;
    t = (int)ceilf((y - f->min_y + r) * g->inv_h);
    const int nMaxCellY = t < ORA_GRID_ROWS - 1 ? t : ORA_GRID_ROWS - 1;
    if (nMaxCellY < 0) return 0;
    const int bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const int c = ix * ORA_GRID_ROWS + iy;
            for (int j = g->start[c]; j < g->start[c + 1]; j++) {
                const ora_keypoint* kp = &f->keys[g->idx[j]];
                if (bCheckLevels) {
                    if (kp->octave < minLevel) continue;
                    if (maxLevel >= 0)
                        if (kp->octave > maxLevel) continue;
                }
                const float distx = kp->x - x;
                const float disty = kp->y - y;
                if (fabsf(distx) < r && fabsf(disty) < r) {
                    if (n < cap) out[n] = g->idx[j];
                    n++;
                }
            }
        }
    }
    return n;
}

/* ---------------------------------------------------------------- helpers */

static int hamming(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 32; i++) d += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    return d;
}

/* ORBmatcher::ComputeThreeMaxima, ORBmatcher.cc:1935-1977 */
void ora_compute_three_maxima(const int* histo_sizes, int L, int* ind1, int* ind2, int* ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = histo_sizes[i];
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            *ind3 = *ind2; *ind2 = *ind1; *ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            *ind3 = *ind2; *ind2 = i;
        } else if (s > max3) {
            max3 = s;
            *ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) {
        *ind2 = -1;
        *ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        *ind3 = -1;
    }
}

/* Rotation-consistency histogram (ORBmatcher.cc:1750-1786): entries are pushed in
 * match order; bins outside the three maxima are un-matched. */
typedef struct {
    int* items[HISTO_LENGTH];
    int size[HISTO_LENGTH];
} rot_hist;

static void hist_init(rot_hist* h, int cap) {
    for (int i = 0; i < HISTO_LENGTH; i++) {
        h->items[i] = (int*)malloc(sizeof(int) * (size_t)(cap + 1));
        h->size[i] = 0;
    }
}

static void hist_free(rot_hist* h) {
    for (int i = 0; i < HISTO_LENGTH; i++) free(h->items[i]);
}

static void hist_push(rot_hist* h, float angle_a, float angle_b, int item) {
    const float factor = HISTO_LENGTH / 360.0f;
    float rot = angle_a - angle_b;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    h->items[bin][h->size[bin]++] = item;
}

static void project(const float* Tcw, const float* X, float* xc) {
    for (int r = 0; r < 3; r++) xc[r] = Tcw[4 * r] * X[0] + Tcw[4 * r + 1] * X[1] + Tcw[4 * r + 2] * X[2] + Tcw[4 * r + 3];
}

/* ---------------------------------------------------------------- a11 */

/* ORBmatcher::RadiusByViewingCos, ORBmatcher.cc:176-183 */
static float radius_by_viewing_cos(float viewCos) { return viewCos > 0.998 ? 2.5f : 4.0f; }

/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th), ORBmatcher.cc:61-173.
 * frame_mp[i]: MapPoint id of keypoint i or -1 (F.mvpMapPoints), updated in place.
 * queries: the vpMapPoints list (MapPoint ids).  Per-MapPoint arrays: descriptor,
 * Observations(), isBad(), and the IsInFrustum outputs (Frame.cc:412-477). */
int ora_sbp_local(const ora_frame* f, int32_t* frame_mp, const int32_t* queries, int nq, const ora_mappoints* mps,
                  const ora_track* trk, float th, float nnratio) {
    ora_grid g;
    ora_grid_build(f, &g);
    int* cand = (int*)malloc(sizeof(int) * (size_t)(f->n + 1));
    int nmatches = 0;
    const int bFactor = th != 1.0;
    for (int iMP = 0; iMP < nq; iMP++) {
        const int mp = queries[iMP];
        if (!trk->in_view[mp]) continue;
        if (mps->bad && mps->bad[mp]) continue;
        const int nPredictedLevel = trk->scale_level[mp];
        float r = radius_by_viewing_cos(trk->view_cos[mp]);
        if (bFactor) r *= th;
        const int nc = ora_features_in_area(f, &g, trk->proj_x[mp], trk->proj_y[mp], r * f->scale_factors[nPredictedLevel],
                                            nPredictedLevel - 1, nPredictedLevel, cand, f->n + 1);
        if (nc == 0) continue;
        const uint8_t* dMP = mps->desc + (size_t)mp * 32;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = cand[c];
            if (frame_mp[idx] >= 0)
                if (mps->observations[frame_mp[idx]] > 0) continue;
            if (f->u_right && f->u_right[idx] > 0) {
                const float er = fabsf(trk->proj_xr[mp] - f->u_right[idx]);
                if (er > r * f->scale_factors[nPredictedLevel]) continue;
            }
            const int dist = hamming(dMP, f->desc + (size_t)idx * 32);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = f->keys[idx].octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = f->keys[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            frame_mp[bestIdx] = mp;
            nmatches++;
        }
    }
    free(cand);
    ora_grid_free(&g);
    return nmatches;
}

/* ---------------------------------------------------------------- a12 */

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, th, bMono),
 * ORBmatcher.cc:1620-1789.  cur_mp in/out; MapPoint arrays give GetWorldPos(),
 * GetDescriptor() and Observations(). */
int ora_sbp_frame(const ora_frame* cur, int32_t* cur_mp, const ora_frame* last, const int32_t* last_mp,
                  const uint8_t* last_outlier, const ora_mappoints* mps, float th, int bMono, int check_ori) {
    ora_grid g;
    ora_grid_build(cur, &g);
    int* cand = (int*)malloc(sizeof(int) * (size_t)(cur->n + 1));
    rot_hist hist;
    hist_init(&hist, cur->n);
    int nmatches = 0;
    /* twc = -Rcw^T tcw; tlc = Rlw*twc + tlw (cc:1637-1643) */
    const float* T = cur->Tcw;
    float twc[3];
    for (int c = 0; c < 3; c++) twc[c] = -(T[c] * T[3] + T[4 + c] * T[7] + T[8 + c] * T[11]);
    float tlc[3];
    project(last->Tcw, twc, tlc);
    const int bForward = tlc[2] > cur->b && !bMono;
    const int bBackward = -tlc[2] > cur->b && !bMono;
    for (int i = 0; i < last->n; i++) {
        const int mp = last_mp[i];
        if (mp < 0) continue;
        if (last_outlier && last_outlier[i]) continue;
        float x3Dc[3];
        project(cur->Tcw, mps->pos + 3 * (size_t)mp, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / x3Dc[2]);
        if (invzc < 0) continue;
        const float u = mad_(cur->fx * xc, invzc, cur->cx);
        const float v = mad_(cur->fy * yc, invzc, cur->cy);
        if (u < cur->min_x || u > cur->max_x) continue;
        if (v < cur->min_y || v > cur->max_y) continue;
        const int nLastOctave = last->keys[i].octave;
        const float radius = th * cur->scale_factors[nLastOctave];
        int nc;
        if (bForward)
            nc = ora_features_in_area(cur, &g, u, v, radius, nLastOctave, -1, cand, cur->n + 1);
        else if (bBackward)
            nc = ora_features_in_area(cur, &g, u, v, radius, 0, nLastOctave, cand, cur->n + 1);
        else
            nc = ora_features_in_area(cur, &g, u, v, radius, nLastOctave - 1, nLastOctave + 1, cand, cur->n + 1);
        if (nc == 0) continue;
        const uint8_t* dMP = mps->desc + (size_t)mp * 32;
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = cand[c];
            if (cur_mp[i2] >= 0)
                if (mps->observations[cur_mp[i2]] > 0) continue;
            if (cur->u_right && cur->u_right[i2] > 0) {
                const float ur = msub_(u, cur->bf, invzc);
                const float er = fabsf(ur - cur->u_right[i2]);
                if (er > radius) continue;
            }
            const int dist = hamming(dMP, cur->desc + (size_t)i2 * 32);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= TH_HIGH) {
            cur_mp[bestIdx2] = mp;
            nmatches++;
            if (check_ori) hist_push(&hist, last->keys[i].angle, cur->keys[bestIdx2].angle, bestIdx2);
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ora_compute_three_maxima(hist.size, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b != ind1 && b != ind2 && b != ind3) {
                for (int j = 0; j < hist.size[b]; j++) {
                    cur_mp[hist.items[b][j]] = -1;
                    nmatches--;
                }
            }
        }
    }
    hist_free(&hist);
    free(cand);
    ora_grid_free(&g);
    return nmatches;
}

/* MapPoint::PredictScale (MapPoint.cc:469-509).  MapPoint.cc has no `using namespace
 * std`, so `log(ratio)` is C's log(double) of the float ratio; the quotient is double and
 * ceil(double).  mfLogScaleFactor = log(mfScaleFactor) (Frame.cc:116, KeyFrame copy),
 * again the double log, stored as float. */
static int predict_scale(float max_distance, float current_dist, const ora_frame* f) {
    const float ratio = max_distance / current_dist;
    const float log_scale = (float)log((double)f->scale_factors[1]);
    int n = (int)ceil(log((double)ratio) / (double)log_scale);
    if (n < 0) n = 0;
    else if (n >= f->nlevels) n = f->nlevels - 1;
    return n;
}

/* cv::norm of a 3x1 CV_32F Mat (NORM_L2): squares accumulated in double, sqrt, to float */
static float norm3(const float* p) {
    double s = 0.0;
    for (int k = 0; k < 3; k++) s += (double)p[k] * p[k];
    return (float)sqrt(s);
}

/* ---------------------------------------------------------------- IsInFrustum */

/* Frame::IsInFrustum(pMP, viewingCosLimit), Frame.cc:412-477, for the MapPoint ids
 * ids[0..n): the Track arrays (indexed by MapPoint id) receive mbTrackInView and, for
 * points in view, mTrackProjX/Y/XR, mnTrackScaleLevel and mTrackViewCos.  Arithmetic as
 * the reference writes it: Pc = Rcw*P + tcw (float products left to right),
 * invz = 1.0f/PcZ in float (Frame.cc:428), the distance bounds 1.2f*mfMaxDistance /
 * 0.8f*mfMinDistance (MapPoint::GetMax/MinDistanceInvariance), cv::norm and Mat::dot in
 * double, viewCos = dot/dist in double stored as float, PredictScale(dist, Frame*). */
void ora_is_in_frustum(const ora_frame* f, const ora_mappoints* mps, const int32_t* ids, int n,
                       float viewingCosLimit, uint8_t* in_view, float* proj_x, float* proj_y, float* proj_xr,
                       int32_t* scale_level, float* view_cos) {
    const float* T = f->Tcw;
    float Ow[3]; /* mOw = -Rcw^T tcw (Frame::UpdatePoseMatrices) */
    for (int c = 0; c < 3; c++) Ow[c] = -(T[c] * T[3] + T[4 + c] * T[7] + T[8 + c] * T[11]);
    for (int k = 0; k < n; k++) {
        const int mp = ids[k];
        in_view[mp] = 0;
        const float* P = mps->pos + 3 * (size_t)mp;
        float Pc[3];
        project(T, P, Pc);
        if (Pc[2] < 0.0f) continue;
        const float invz = 1.0f / Pc[2];
        const float u = mad_(f->fx * Pc[0], invz, f->cx);
        const float v = mad_(f->fy * Pc[1], invz, f->cy);
        if (u < f->min_x || u > f->max_x) continue;
        if (v < f->min_y || v > f->max_y) continue;
        const float maxDistance = 1.2f * mps->max_distance[mp];
        const float minDistance = 0.8f * mps->min_distance[mp];
        float PO[3];
        for (int c = 0; c < 3; c++) PO[c] = P[c] - Ow[c];
        const float dist = norm3(PO);
        if (dist < minDistance || dist > maxDistance) continue;
        const float* Pn = mps->normal + 3 * (size_t)mp;
        double dot = 0.0;
        for (int c = 0; c < 3; c++) dot += (double)PO[c] * Pn[c];
        const float viewCos = (float)(dot / dist);
        if (viewCos < viewingCosLimit) continue;
        in_view[mp] = 1;
        proj_x[mp] = u;
        proj_xr[mp] = msub_(u, f->bf, invz);
        proj_y[mp] = v;
        scale_level[mp] = predict_scale(mps->max_distance[mp], dist, f);
        view_cos[mp] = viewCos;
    }
}

/* ---------------------------------------------------------------- MapPoint creation */

/* Tracking::CreateNewKeyFrame's MapPoints of one Frame (Tracking.cc:1069-1121): keypoint
 * i with depth z > 0 (depth[i], or const_depth when depth is NULL) gets
 * Frame::UnprojectStereo(i) (Frame.cc:912-927: x3Dc = ((u-cx)*z*invfx, (v-cy)*z*invfy, z),
 * mRwc*x3Dc + mOw) and MapPoint::UpdateNormalAndDepth with this frame as its only
 * observation (MapPoint.cc:386-439: normal = PC / cv::norm(PC), i.e. PC * (float)(1/n);
 * mfMaxDistance = |PC| * mvScaleFactors[octave]; mfMinDistance = mfMaxDistance /
 * mvScaleFactors[nLevels-1]).  valid[i] = 0 where no MapPoint is made. */
void ora_create_mappoints(const ora_frame* f, const float* depth, float const_depth, float* pos, float* normal,
                          float* max_distance, float* min_distance, uint8_t* valid) {
    const float* T = f->Tcw;
    const float invfx = 1.0f / f->fx, invfy = 1.0f / f->fy;
    float Ow[3];
    for (int r = 0; r < 3; r++) Ow[r] = -(T[r] * T[3] + T[4 + r] * T[7] + T[8 + r] * T[11]);
    for (int i = 0; i < f->n; i++) {
        const float z = depth ? depth[i] : const_depth;
        valid[i] = 0;
        if (!(z > 0)) continue;
        const float x = (f->keys[i].x - f->cx) * z * invfx;
        const float y = (f->keys[i].y - f->cy) * z * invfy;
        float P[3], PC[3];
        for (int r = 0; r < 3; r++) P[r] = T[r] * x + T[4 + r] * y + T[8 + r] * z + Ow[r];
        for (int c = 0; c < 3; c++) PC[c] = P[c] - Ow[c];
        const double n = sqrt((double)PC[0] * PC[0] + (double)PC[1] * PC[1] + (double)PC[2] * PC[2]);
        const float inv = (float)(1.0 / n);
        const float dist = (float)n;
        int oct = f->keys[i].octave;
        if (oct < 0) oct = 0;
        if (oct >= f->nlevels) oct = f->nlevels - 1;
        const float mx = dist * f->scale_factors[oct];
        for (int c = 0; c < 3; c++) {
            pos[3 * i + c] = P[c];
            normal[3 * i + c] = PC[c] * inv;
        }
        max_distance[i] = mx;
        min_distance[i] = mx / f->scale_factors[f->nlevels - 1];
        valid[i] = 1;
    }
}

/* Tracking::UpdateLastFrame (Tracking.cc:893-954), after SetPose, for a stereo / RGB-D
 * LastFrame that is not the last keyframe: the pairs (mvDepth[i], i) with depth > 0 are
 * sorted ascending (std::sort of pair<float,int>: depth, then index) and visited in order;
 * a keypoint without a MapPoint, or whose MapPoint has Observations() < 1, gets a new
 * temporal MapPoint at Frame::UnprojectStereo(i) (created without AddObservation, so its
 * Observations() is 0); every visited point counts, and the walk stops after the first
 * point deeper than th_depth (mThDepth) once more than 100 have been visited (cc:951-952).
 * mp_obs[i]: in, Observations() of keypoint i's MapPoint (-1 = NULL); out, 0 where a
 * temporal point was made.  pos[3i..3i+2]: in, that MapPoint's GetWorldPos(); out, the
 * temporal point's.  Returns the number of temporal points. */
typedef struct {
    float z;
    int i;
} depth_idx;

static int cmp_depth_idx(const void* a, const void* b) {
    const depth_idx* x = (const depth_idx*)a;
    const depth_idx* y = (const depth_idx*)b;
    if (x->z < y->z) return -1;
    if (x->z > y->z) return 1;
    return (x->i > y->i) - (x->i < y->i);
}

int ora_update_last_frame(const ora_frame* f, const float* depth, float th_depth, int32_t* mp_obs, float* pos) {
    depth_idx* v = (depth_idx*)malloc(sizeof(depth_idx) * (size_t)(f->n + 1));
    int m = 0;
    for (int i = 0; i < f->n; i++)
        if (depth[i] > 0) {
            v[m].z = depth[i];
            v[m].i = i;
            m++;
        }
    qsort(v, (size_t)m, sizeof(depth_idx), cmp_depth_idx);
    const float* T = f->Tcw;
    const float invfx = 1.0f / f->fx, invfy = 1.0f / f->fy;
    float Ow[3];
    for (int r = 0; r < 3; r++) Ow[r] = -(T[r] * T[3] + T[4 + r] * T[7] + T[8 + r] * T[11]);
    int nPoints = 0, created = 0;
    for (int j = 0; j < m; j++) {
        const int i = v[j].i;
        if (mp_obs[i] < 1) { /* !pMP || pMP->Observations() < 1 */
            const float z = depth[i];
            const float x = (f->keys[i].x - f->cx) * z * invfx;
            const float y = (f->keys[i].y - f->cy) * z * invfy;
            for (int r = 0; r < 3; r++) pos[3 * i + r] = T[r] * x + T[4 + r] * y + T[8 + r] * z + Ow[r];
            mp_obs[i] = 0;
            created++;
        }
        nPoints++;
        if (v[j].z > th_depth && nPoints > 100) break;
    }
    free(v);
    return created;
}

/* ---------------------------------------------------------------- a13 */

/* ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>&
 * sAlreadyFound, th, ORBdist), ORBmatcher.cc:1792-1924.  kf_mp: pKF->GetMapPointMatches()
 * as ids; already_found[id] or NULL.  Claims: any assigned keypoint is skipped
 * (cc:1865-1866). */
int ora_sbp_keyframe(const ora_frame* cur, int32_t* cur_mp, const ora_frame* kf, const int32_t* kf_mp,
                     const uint8_t* already_found, const ora_mappoints* mps, float th, int orb_dist, int check_ori) {
    ora_grid g;
    ora_grid_build(cur, &g);
    int* cand = (int*)malloc(sizeof(int) * (size_t)(cur->n + 1));
    rot_hist hist;
    hist_init(&hist, cur->n);
    int nmatches = 0;
    const float* T = cur->Tcw;
    float Ow[3];  /* -Rcw^T tcw (cc:1796-1798) */
    for (int c = 0; c < 3; c++) Ow[c] = -(T[c] * T[3] + T[4 + c] * T[7] + T[8 + c] * T[11]);
    for (int i = 0; i < kf->n; i++) {
        const int mp = kf_mp[i];
        if (mp < 0) continue;
        if (mps->bad && mps->bad[mp]) continue;
        if (already_found && already_found[mp]) continue;
        const float* x3Dw = mps->pos + 3 * (size_t)mp;
        float x3Dc[3];
        project(cur->Tcw, x3Dw, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / x3Dc[2]);
        const float u = mad_(cur->fx * xc, invzc, cur->cx);
        const float v = mad_(cur->fy * yc, invzc, cur->cy);
        if (u < cur->min_x || u > cur->max_x) continue;
        if (v < cur->min_y || v > cur->max_y) continue;
        float PO[3];
        for (int c = 0; c < 3; c++) PO[c] = x3Dw[c] - Ow[c];
        const float dist3D = norm3(PO);
        const float maxDistance = 1.2f * mps->max_distance[mp];
        const float minDistance = 0.8f * mps->min_distance[mp];
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int nPredictedLevel = predict_scale(mps->max_distance[mp], dist3D, cur);
        const float radius = th * cur->scale_factors[nPredictedLevel];
        const int nc = ora_features_in_area(cur, &g, u, v, radius, nPredictedLevel - 1, nPredictedLevel + 1, cand,
                                            cur->n + 1);
        if (nc == 0) continue;
        const uint8_t* dMP = mps->desc + (size_t)mp * 32;
        int bestDist = 256, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = cand[c];
            if (cur_mp[i2] >= 0) continue;
            const int dist = hamming(dMP, cur->desc + (size_t)i2 * 32);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = i2;
            }
        }
        if (bestDist <= orb_dist) {
            cur_mp[bestIdx2] = mp;
            nmatches++;
            if (check_ori) hist_push(&hist, kf->keys[i].angle, cur->keys[bestIdx2].angle, bestIdx2);
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ora_compute_three_maxima(hist.size, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b != ind1 && b != ind2 && b != ind3) {
                for (int j = 0; j < hist.size[b]; j++) {
                    cur_mp[hist.items[b][j]] = -1;
                    nmatches--;
                }
            }
        }
    }
    hist_free(&hist);
    free(cand);
    ora_grid_free(&g);
    return nmatches;
}

/* ---------------------------------------------------------------- a14 */

/* ORBmatcher::SearchByProjection(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>&
 * vpPoints, vector<MapPoint*>& vpMatched, int th), ORBmatcher.cc:398-520.  Scw 3x4
 * row-major.  OpenCV arithmetic as restated: Mat::dot accumulates in
 * double; Mat / scalar multiplies by (float)(1/s); Mat products sum float products left
 * to right. */
int ora_sbp_sim3(const ora_frame* kf, const float* Scw, const int32_t* points, int npoints, int32_t* matched,
                 const ora_mappoints* mps, int th) {
    ora_grid g;
    ora_grid_build(kf, &g);
    int* cand = (int*)malloc(sizeof(int) * (size_t)(kf->n + 1));
    double d0 = 0.0;
    for (int c = 0; c < 3; c++) d0 += (double)Scw[c] * Scw[c];
    const float scw = (float)sqrt(d0);
    const float alpha = (float)(1.0 / scw);
    float T[12];  /* [Rcw | tcw] */
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) T[4 * r + c] = Scw[4 * r + c] * alpha;
    float Ow[3];
    for (int c = 0; c < 3; c++) Ow[c] = -(T[c] * T[3] + T[4 + c] * T[7] + T[8 + c] * T[11]);
    /* spAlreadyFound: the MapPoints of vpMatched before the loop */
    uint8_t* found = (uint8_t*)calloc((size_t)(mps->n > 0 ? mps->n : 1), 1);
    for (int i = 0; i < kf->n; i++)
        if (matched[i] >= 0) found[matched[i]] = 1;
    int nmatches = 0;
    for (int k = 0; k < npoints; k++) {
        const int mp = points[k];
        if ((mps->bad && mps->bad[mp]) || found[mp]) continue;
        const float* p3Dw = mps->pos + 3 * (size_t)mp;
        float p3Dc[3];
        project(T, p3Dw, p3Dc);
        if (p3Dc[2] < 0.0) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz;
        const float y = p3Dc[1] * invz;
        const float u = mad_(kf->fx, x, kf->cx);
        const float v = mad_(kf->fy, y, kf->cy);
        if (!(u >= kf->min_x && u < kf->max_x && v >= kf->min_y && v < kf->max_y)) continue;  /* IsInImage */
        const float maxDistance = 1.2f * mps->max_distance[mp];
        const float minDistance = 0.8f * mps->min_distance[mp];
        float PO[3];
        for (int c = 0; c < 3; c++) PO[c] = p3Dw[c] - Ow[c];
        const float dist = norm3(PO);
        if (dist < minDistance || dist > maxDistance) continue;
        const float* Pn = mps->normal + 3 * (size_t)mp;
        double dot = 0.0;
        for (int c = 0; c < 3; c++) dot += (double)PO[c] * Pn[c];
        if (dot < 0.5 * dist) continue;
        const int nPredictedLevel = predict_scale(mps->max_distance[mp], dist, kf);
        const float radius = th * kf->scale_factors[nPredictedLevel];
        const int nc = ora_features_in_area(kf, &g, u, v, radius, -1, -1, cand, kf->n + 1);
        if (nc == 0) continue;
        const uint8_t* dMP = mps->desc + (size_t)mp * 32;
        int bestDist = 256, bestIdx = -1;
        for (int c = 0; c < nc; c++) {
            const int idx = cand[c];
            if (matched[idx] >= 0) continue;
            const int kpLevel = kf->keys[idx].octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const int d = hamming(dMP, kf->desc + (size_t)idx * 32);
            if (d < bestDist) {
                bestDist = d;
                bestIdx = idx;
            }
        }
        if (bestDist <= TH_LOW) {
            matched[bestIdx] = mp;
            nmatches++;
        }
    }
    free(found);
    free(cand);
    ora_grid_free(&g);
    return nmatches;
}

/* ---------------------------------------------------------------- a15 */

/* ORBmatcher::CheckDistEpipolarLine, ORBmatcher.cc:186-213 */
static int check_dist_epipolar_line(const ora_keypoint* kp1, const ora_keypoint* kp2, const float* F12,
                                    const float* sigma2) {
    const float a = mad_(kp1->x, F12[0], kp1->y * F12[3]) + F12[6];
    const float b = mad_(kp1->x, F12[1], kp1->y * F12[4]) + F12[7];
    const float c = mad_(kp1->x, F12[2], kp1->y * F12[5]) + F12[8];
    const float num = mad_(a, kp2->x, b * kp2->y) + c;
    const float den = mad_(a, a, b * b);
    if (den == 0) return 0;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * sigma2[kp2->octave];
}

/* ORBmatcher::SearchForTriangulation, ORBmatcher.cc:850-1056.  kf*_has_mp[i]: the
 * keyframe keypoint already has a MapPoint.  FeatureVectors as CSR: fv*_node[k]
 * (ascending node ids), keypoints of node k at fv*_idx[fv*_off[k] .. fv*_off[k+1]).
 * F12 row-major 3x3.  Writes pairs (idx1, idx2) in idx1 order; returns the count. */
int ora_search_for_triangulation(const ora_frame* kf1, const uint8_t* kf1_has_mp, const int32_t* fv1_node,
                                 const int32_t* fv1_off, const int32_t* fv1_idx, int fv1_n, const ora_frame* kf2,
                                 const uint8_t* kf2_has_mp, const int32_t* fv2_node, const int32_t* fv2_off,
                                 const int32_t* fv2_idx, int fv2_n, const float* F12, int bOnlyStereo,
                                 int check_ori, int32_t* pairs /* 2*kf1->n */) {
    /* Cw = KF1 camera centre = -R1^T t1; C2 = R2w*Cw + t2w (cc:858-865) */
    const float* T1 = kf1->Tcw;
    float Cw[3];
    for (int c = 0; c < 3; c++) Cw[c] = -(T1[c] * T1[3] + T1[4 + c] * T1[7] + T1[8 + c] * T1[11]);
    float C2[3];
    project(kf2->Tcw, Cw, C2);
    const float invz = 1.0f / C2[2];
    const float ex = mad_(kf2->fx * C2[0], invz, kf2->cx);
    const float ey = mad_(kf2->fy * C2[1], invz, kf2->cy);

    uint8_t* vbMatched2 = (uint8_t*)calloc((size_t)kf2->n + 1, 1);
    int32_t* vMatches12 = (int32_t*)malloc(sizeof(int32_t) * (size_t)(kf1->n + 1));
    for (int i = 0; i < kf1->n; i++) vMatches12[i] = -1;
    rot_hist hist;
    hist_init(&hist, kf1->n);
    int nmatches = 0;
    int f1 = 0, f2 = 0;
    while (f1 < fv1_n && f2 < fv2_n) {
        if (fv1_node[f1] == fv2_node[f2]) {
            for (int i1 = fv1_off[f1]; i1 < fv1_off[f1 + 1]; i1++) {
                const int idx1 = fv1_idx[i1];
                if (kf1_has_mp[idx1]) continue;
                const int bStereo1 = kf1->u_right && kf1->u_right[idx1] >= 0;
                if (bOnlyStereo && !bStereo1) continue;
                const ora_keypoint* kp1 = &kf1->keys[idx1];
                const uint8_t* d1 = kf1->desc + (size_t)idx1 * 32;
                int bestDist = TH_LOW, bestIdx2 = -1;
                for (int i2 = fv2_off[f2]; i2 < fv2_off[f2 + 1]; i2++) {
                    const int idx2 = fv2_idx[i2];
                    if (vbMatched2[idx2] || kf2_has_mp[idx2]) continue;
                    const int bStereo2 = kf2->u_right && kf2->u_right[idx2] >= 0;
                    if (bOnlyStereo && !bStereo2) continue;
                    const int dist = hamming(d1, kf2->desc + (size_t)idx2 * 32);
                    if (dist > TH_LOW || dist > bestDist) continue;
                    const ora_keypoint* kp2 = &kf2->keys[idx2];
                    if (!bStereo1 && !bStereo2) {
                        const float distex = ex - kp2->x;
                        const float distey = ey - kp2->y;
                        if (mad_(distex, distex, distey * distey) < 100 * kf2->scale_factors[kp2->octave]) continue;
                    }
                    if (check_dist_epipolar_line(kp1, kp2, F12, kf2->level_sigma2)) {
                        bestIdx2 = idx2;
                        bestDist = dist;
                    }
                }
                if (bestIdx2 >= 0) {
                    vMatches12[idx1] = bestIdx2;
                    vbMatched2[bestIdx2] = 1;
                    nmatches++;
                    if (check_ori) hist_push(&hist, kp1->angle, kf2->keys[bestIdx2].angle, idx1);
                }
            }
            f1++;
            f2++;
        } else if (fv1_node[f1] < fv2_node[f2]) {
            while (f1 < fv1_n && fv1_node[f1] < fv2_node[f2]) f1++;  /* lower_bound */
        } else {
            while (f2 < fv2_n && fv2_node[f2] < fv1_node[f1]) f2++;
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ora_compute_three_maxima(hist.size, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int j = 0; j < hist.size[b]; j++) {
                vMatches12[hist.items[b][j]] = -1;
                nmatches--;
            }
        }
    }
    int np = 0;
    for (int i = 0; i < kf1->n; i++) {
        if (vMatches12[i] < 0) continue;
        pairs[2 * np] = i;
        pairs[2 * np + 1] = vMatches12[i];
        np++;
    }
    hist_free(&hist);
    free(vbMatched2);
    free(vMatches12);
    return np;
}

/* ---------------------------------------------------------------- a18 */

/* Frame::ComputeStereoMatches, Frame.cc:673-885, this fork's semantics: the
 * median-based outlier pass runs inside the per-keypoint loop (after every left
 * keypoint that is not skipped by a `continue`), on the entries collected so far;
 * an empty list is skipped (the reference reads vDistIdx[0] of an empty vector,
 * whose value cannot matter because the marking loop then runs zero times).
 * maxD is passed explicitly: the fork computes mbf/mb with mb not yet set
 * (Frame.cc:711-713, mb is assigned at Frame.cc:174); upstream's value is fx.
 * levels_l/levels_r: pyramid level ROIs (w_l x h_l, row stride w_l). */
void ora_compute_stereo_matches(const ora_frame* left, const ora_keypoint* keys_r, const uint8_t* desc_r, int nr,
                                const uint8_t* const* levels_l, const uint8_t* const* levels_r, const int* level_w,
                                const int* level_h, const float* inv_scale, float maxD, float* u_right,
                                float* depth) {
    const int N = left->n;
    for (int i = 0; i < N; i++) u_right[i] = -1.0f, depth[i] = -1.0f;
    const int thOrbDist = (TH_HIGH + TH_LOW) / 2;
    const int nRows = level_h[0];
    /* vRowIndices: right keypoint indices per image row (cc:693-708) */
    int* rcnt = (int*)calloc((size_t)nRows + 1, sizeof(int));
    for (int pass = 0; pass < 2; pass++) {
        for (int iR = 0; iR < nr; iR++) {
            const float kpY = keys_r[iR].y;
            const float r = 2.0f * left->scale_factors[keys_r[iR].octave];
            const int maxr = (int)ceilf(kpY + r);
            const int minr = (int)floorf(kpY - r);
            for (int yi = minr; yi <= maxr; yi++) {
                if (yi < 0 || yi >= nRows) continue; /* never happens for keypoints >= 19 px from the border */
                if (pass == 0) rcnt[yi + 1]++;
            }
        }
        if (pass == 0)
            for (int y = 0; y < nRows; y++) rcnt[y + 1] += rcnt[y];
    }
    int* rows = (int*)malloc(sizeof(int) * (size_t)(rcnt[nRows] + 1));
    int* fill = (int*)calloc((size_t)nRows, sizeof(int));
    for (int iR = 0; iR < nr; iR++) {
        const float kpY = keys_r[iR].y;
        const float r = 2.0f * left->scale_factors[keys_r[iR].octave];
        const int maxr = (int)ceilf(kpY + r);
        const int minr = (int)floorf(kpY - r);
        for (int yi = minr; yi <= maxr; yi++)
            if (yi >= 0 && yi < nRows) rows[rcnt[yi] + fill[yi]++] = iR;
    }
    const float minD = 0;
    /* vDistIdx as (dist, iL) pairs kept sorted */
    int* vd = (int*)malloc(sizeof(int) * 2 * (size_t)(N + 1));
    int nvd = 0;
    for (int iL = 0; iL < N; iL++) {
        const ora_keypoint* kpL = &left->keys[iL];
        const int levelL = kpL->octave;
        const float vL = kpL->y, uL = kpL->x;
        const int row = (int)vL;
        if (rcnt[row + 1] - rcnt[row] == 0) continue;
        const float minU = uL - maxD;
        const float maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = TH_HIGH;
        int bestIdxR = 0;
        const uint8_t* dL = left->desc + (size_t)iL * 32;
        for (int c = rcnt[row]; c < rcnt[row + 1]; c++) {
            const int iR = rows[c];
            const ora_keypoint* kpR = &keys_r[iR];
            if (kpR->octave < levelL - 1 || kpR->octave > levelL + 1) continue;
            const float uR = kpR->x;
            if (uR >= minU && uR <= maxU) {
                const int dist = hamming(dL, desc_r + (size_t)iR * 32);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist < thOrbDist) {
            const float uR0 = keys_r[bestIdxR].x;
            const float scaleFactor = inv_scale[levelL];
            const float scaleduL = roundf(kpL->x * scaleFactor);
            const float scaledvL = roundf(kpL->y * scaleFactor);
            const float scaleduR0 = roundf(uR0 * scaleFactor);
            const int w = 5, L = 5;
            const int lw = level_w[levelL];
            const uint8_t* IL = levels_l[levelL];
            const uint8_t* IR = levels_r[levelL];
            const int yl0 = (int)scaledvL - w, xl0 = (int)scaleduL - w;
            const float cl = (float)IL[(size_t)(yl0 + w) * lw + xl0 + w];
            int bestDistS = INT_MAX;
            int bestincR = 0;
            float vDists[11];
            const float iniu = scaleduR0 + L - w;
            const float endu = scaleduR0 + L + w + 1;
            if (iniu < 0 || endu >= level_w[levelL]) continue;
            for (int incR = -L; incR <= +L; incR++) {
                const int xr0 = (int)(scaleduR0 + incR - w);
                const float cr = (float)IR[(size_t)(yl0 + w) * lw + xr0 + w];
                double acc = 0;
                for (int yy = 0; yy < 2 * w + 1; yy++)
                    for (int xx = 0; xx < 2 * w + 1; xx++) {
                        const float a = (float)IL[(size_t)(yl0 + yy) * lw + xl0 + xx] - cl;
                        const float b = (float)IR[(size_t)(yl0 + yy) * lw + xr0 + xx] - cr;
                        acc += fabs((double)a - (double)b);
                    }
                const float dist = (float)acc;  /* cv::norm(IL, IR, NORM_L1) */
                if (dist < bestDistS) {
                    bestDistS = (int)dist;
                    bestincR = incR;
                }
                vDists[L + incR] = dist;
            }
            if (bestincR == -L || bestincR == L) continue;
            const float dist1 = vDists[L + bestincR - 1];
            const float dist2 = vDists[L + bestincR];
            const float dist3 = vDists[L + bestincR + 1];
            const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
            if (deltaR < -1 || deltaR > 1) continue;
            float bestuR = left->scale_factors[levelL] * (scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < maxD) {
                if (disparity <= 0) {
                    disparity = 0.01f;
                    bestuR = (float)(uL - 0.01);
                }
                depth[iL] = left->bf / disparity;
                u_right[iL] = bestuR;
                /* insert (bestDistS, iL) keeping (dist, idx) order */
                int pos = nvd;
                while (pos > 0 && (vd[2 * (pos - 1)] > bestDistS ||
                                   (vd[2 * (pos - 1)] == bestDistS && vd[2 * (pos - 1) + 1] > iL))) {
                    vd[2 * pos] = vd[2 * (pos - 1)];
                    vd[2 * pos + 1] = vd[2 * (pos - 1) + 1];
                    pos--;
                }
                vd[2 * pos] = bestDistS;
                vd[2 * pos + 1] = iL;
                nvd++;
            }
        }
        /* outlier pass inside the loop (Frame.cc:868-884) */
        if (nvd > 0) {
            const float median = (float)vd[2 * (nvd / 2)];
            const float thDist = 1.5f * 1.4f * median;
            for (int i = nvd - 1; i >= 0; i--) {
                if ((float)vd[2 * i] < thDist) break;
                u_right[vd[2 * i + 1]] = -1;
                depth[vd[2 * i + 1]] = -1;
            }
        }
    }
    free(vd);
    free(rows);
    free(fill);
    free(rcnt);
}

/* ---------------------------------------------------------------- f2 */

/* ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&), ORBmatcher.cc:228-392.
 * kf_mp[i]: MapPoint id of KF keypoint i, -1 when NULL or isBad().  FeatureVectors as
 * CSR (see ora_search_for_triangulation).  matches[f->n] out: the KF MapPoint id matched
 * to each frame keypoint or -1.  The histogram uses the frame keypoint's angle from
 * mvKeys (== mvKeysUn's angle). */
int ora_search_by_bow_kf_frame(const ora_frame* kf, const int32_t* kf_mp, const int32_t* fv1_node,
                               const int32_t* fv1_off, const int32_t* fv1_idx, int fv1_n, const ora_frame* f,
                               const int32_t* fv2_node, const int32_t* fv2_off, const int32_t* fv2_idx, int fv2_n,
                               float nnratio, int check_ori, int32_t* matches) {
    for (int i = 0; i < f->n; i++) matches[i] = -1;
    rot_hist hist;
    hist_init(&hist, f->n);
    int nmatches = 0;
    int f1 = 0, f2 = 0;
    while (f1 < fv1_n && f2 < fv2_n) {
        if (fv1_node[f1] == fv2_node[f2]) {
            for (int i1 = fv1_off[f1]; i1 < fv1_off[f1 + 1]; i1++) {
                const int realIdxKF = fv1_idx[i1];
                const int pMP = kf_mp[realIdxKF];
                if (pMP < 0) continue;
                const uint8_t* dKF = kf->desc + (size_t)realIdxKF * 32;
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                for (int i2 = fv2_off[f2]; i2 < fv2_off[f2 + 1]; i2++) {
                    const int realIdxF = fv2_idx[i2];
                    if (matches[realIdxF] >= 0) continue;
                    const int dist = hamming(dKF, f->desc + (size_t)realIdxF * 32);
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1;
                        bestDist1 = dist;
                        bestIdxF = realIdxF;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 <= TH_LOW) {
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        matches[bestIdxF] = pMP;
                        if (check_ori) hist_push(&hist, kf->keys[realIdxKF].angle, f->keys[bestIdxF].angle, bestIdxF);
                        nmatches++;
                    }
                }
            }
            f1++;
            f2++;
        } else if (fv1_node[f1] < fv2_node[f2]) {
            while (f1 < fv1_n && fv1_node[f1] < fv2_node[f2]) f1++;
        } else {
            while (f2 < fv2_n && fv2_node[f2] < fv1_node[f1]) f2++;
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ora_compute_three_maxima(hist.size, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int j = 0; j < hist.size[b]; j++) {
                matches[hist.items[b][j]] = -1;
                nmatches--;
            }
        }
    }
    hist_free(&hist);
    return nmatches;
}

/* ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&), ORBmatcher.cc:696-839.
 * mp1 / mp2: MapPoint ids (-1 = NULL or bad).  matches12[kf1->n] out: KF2's MapPoint
 * id matched to each KF1 keypoint or -1. */
int ora_search_by_bow_kf_kf(const ora_frame* kf1, const int32_t* mp1, const int32_t* fv1_node, const int32_t* fv1_off,
                            const int32_t* fv1_idx, int fv1_n, const ora_frame* kf2, const int32_t* mp2,
                            const int32_t* fv2_node, const int32_t* fv2_off, const int32_t* fv2_idx, int fv2_n,
                            float nnratio, int check_ori, int32_t* matches12) {
    for (int i = 0; i < kf1->n; i++) matches12[i] = -1;
    uint8_t* vbMatched2 = (uint8_t*)calloc((size_t)kf2->n + 1, 1);
    rot_hist hist;
    hist_init(&hist, kf1->n);
    int nmatches = 0;
    int f1 = 0, f2 = 0;
    while (f1 < fv1_n && f2 < fv2_n) {
        if (fv1_node[f1] == fv2_node[f2]) {
            for (int i1 = fv1_off[f1]; i1 < fv1_off[f1 + 1]; i1++) {
                const int idx1 = fv1_idx[i1];
                if (mp1[idx1] < 0) continue;
                const uint8_t* d1 = kf1->desc + (size_t)idx1 * 32;
                int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
                for (int i2 = fv2_off[f2]; i2 < fv2_off[f2 + 1]; i2++) {
                    const int idx2 = fv2_idx[i2];
                    if (vbMatched2[idx2] || mp2[idx2] < 0) continue;
                    const int dist = hamming(d1, kf2->desc + (size_t)idx2 * 32);
                    if (dist < bestDist1) {
                        bestDist2 = bestDist1;
                        bestDist1 = dist;
                        bestIdx2 = idx2;
                    } else if (dist < bestDist2) {
                        bestDist2 = dist;
                    }
                }
                if (bestDist1 < TH_LOW) {
                    if ((float)bestDist1 < nnratio * (float)bestDist2) {
                        matches12[idx1] = mp2[bestIdx2];
                        vbMatched2[bestIdx2] = 1;
                        if (check_ori) hist_push(&hist, kf1->keys[idx1].angle, kf2->keys[bestIdx2].angle, idx1);
                        nmatches++;
                    }
                }
            }
            f1++;
            f2++;
        } else if (fv1_node[f1] < fv2_node[f2]) {
            while (f1 < fv1_n && fv1_node[f1] < fv2_node[f2]) f1++;
        } else {
            while (f2 < fv2_n && fv2_node[f2] < fv1_node[f1]) f2++;
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ora_compute_three_maxima(hist.size, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int j = 0; j < hist.size[b]; j++) {
                matches12[hist.items[b][j]] = -1;
                nmatches--;
            }
        }
    }
    hist_free(&hist);
    free(vbMatched2);
    return nmatches;
}

/* ORBmatcher::SearchForInitialization, ORBmatcher.cc:539-683.  prev_matched[2*n1]
 * (vbPrevMatched) in/out; matches12[f1->n] out (vnMatches12). */
int ora_search_for_initialization(const ora_frame* f1, const ora_frame* f2, float* prev_matched, int32_t* matches12,
                                  int windowSize, float nnratio, int check_ori) {
    int nmatches = 0;
    for (int i = 0; i < f1->n; i++) matches12[i] = -1;
    rot_hist hist;
    hist_init(&hist, f1->n);
    ora_grid g;
    ora_grid_build(f2, &g);
    int* vMatchedDistance = (int*)malloc(sizeof(int) * (size_t)(f2->n + 1));
    int* vnMatches21 = (int*)malloc(sizeof(int) * (size_t)(f2->n + 1));
    int* cand = (int*)malloc(sizeof(int) * (size_t)(f2->n + 1));
    for (int i = 0; i < f2->n; i++) {
        vMatchedDistance[i] = 0x7fffffff;
        vnMatches21[i] = -1;
    }
    for (int i1 = 0; i1 < f1->n; i1++) {
        const ora_keypoint* kp1 = &f1->keys[i1];
        const int level1 = kp1->octave;
        if (level1 > 0) continue;
        const int nc = ora_features_in_area(f2, &g, prev_matched[2 * i1], prev_matched[2 * i1 + 1], (float)windowSize,
                                            level1, level1, cand, f2->n + 1);
        if (nc == 0) continue;
        const uint8_t* d1 = f1->desc + (size_t)i1 * 32;
        int bestDist = 0x7fffffff, bestDist2 = 0x7fffffff, bestIdx2 = -1;
        for (int c = 0; c < nc; c++) {
            const int i2 = cand[c];
            const int dist = hamming(d1, f2->desc + (size_t)i2 * 32);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) {
                    matches12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                matches12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (check_ori) hist_push(&hist, f1->keys[i1].angle, f2->keys[bestIdx2].angle, i1);
            }
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        ora_compute_three_maxima(hist.size, HISTO_LENGTH, &ind1, &ind2, &ind3);
        for (int b = 0; b < HISTO_LENGTH; b++) {
            if (b == ind1 || b == ind2 || b == ind3) continue;
            for (int j = 0; j < hist.size[b]; j++) {
                const int idx1 = hist.items[b][j];
                if (matches12[idx1] >= 0) {
                    matches12[idx1] = -1;
                    nmatches--;
                }
            }
        }
    }
    for (int i1 = 0; i1 < f1->n; i1++)
        if (matches12[i1] >= 0) {
            prev_matched[2 * i1] = f2->keys[matches12[i1]].x;
            prev_matched[2 * i1 + 1] = f2->keys[matches12[i1]].y;
        }
    free(cand);
    free(vnMatches21);
    free(vMatchedDistance);
    ora_grid_free(&g);
    hist_free(&hist);
    return nmatches;
}

/* ---------------------------------------------------------------- f3 */

/* cv::undistortPoints(src, dst, K, D, noArray(), K) for CV_32FC2 points, OpenCV 3.3.1
 * cvUndistortPoints (imgproc/src/undistort.cpp, not vendored: parity unpinned), as
 * called by Frame::UndistortKeyPoints (Frame.cc:586-628) and ComputeImageBounds
 * (Frame.cc:636-665).  K = (fx, fy, cx, cy), D = (k1, k2, p1, p2, k3), all converted to
 * double; 5 fixed-point iterations; R = I and P = K make the final projection
 * fx*x + cx exactly; the result is rounded to float. */
void ora_undistort_points(const float* K, const float* D, const float* pts, int n, float* out) {
    const double fx = K[0], fy = K[1], cx = K[2], cy = K[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    double k[14] = {0};
    for (int i = 0; i < 5; i++) k[i] = D[i];
    for (int i = 0; i < n; i++) {
        double x = pts[2 * i], y = pts[2 * i + 1];
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; j++) {
            const double r2 = x * x + y * y;
            const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
            const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        const double xx = fx * x + 0. * y + cx;
        const double yy = 0. * x + fy * y + cy;
        const double ww = 1. / (0. * x + 0. * y + 1.);
        out[2 * i] = (float)(xx * ww);
        out[2 * i + 1] = (float)(yy * ww);
    }
}

/* ---------------------------------------------------------------- f4 */

/* Window search shared by Fuse / SearchBySim3: the first keypoint (GetFeaturesInArea
 * order) with the smallest distance among those with octave in [pred-1, pred] (and,
 * when gate, inside Fuse's chi-square gate); returns it when its distance <= accept. */
static int window_best(const ora_frame* kf, const ora_grid* g, int* cand, const uint8_t* dMP, float u, float v,
                       float ur, float radius, int pred, int gate, const float* inv_sigma2, int accept) {
    const int nc = ora_features_in_area(kf, g, u, v, radius, -1, -1, cand, kf->n + 1);
    if (nc == 0) return -1;
    int bestDist = 256, bestIdx = -1;
    for (int c = 0; c < nc; c++) {
        const int idx = cand[c];
        const ora_keypoint* kp = &kf->keys[idx];
        const int kpLevel = kp->octave;
        if (kpLevel < pred - 1 || kpLevel > pred) continue;
        if (gate) {
            if (kf->u_right && kf->u_right[idx] >= 0) { /* cc:1137-1150 */
                const float ex = u - kp->x, ey = v - kp->y, er = ur - kf->u_right[idx];
                const float e2 = mad_(er, er, mad_(ex, ex, ey * ey));
                if ((double)(e2 * inv_sigma2[kpLevel]) > 7.8) continue;
            } else {
                const float ex = u - kp->x, ey = v - kp->y;
                const float e2 = mad_(ex, ex, ey * ey);
                if ((double)(e2 * inv_sigma2[kpLevel]) > 5.99) continue;
            }
        }
        const int d = hamming(dMP, kf->desc + (size_t)idx * 32);
        if (d < bestDist) {
            bestDist = d;
            bestIdx = idx;
        }
    }
    return bestDist <= accept ? bestIdx : -1;
}

/* ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, th),
 * ORBmatcher.cc:1067-1221: the search part.  points[k]: MapPoint id or -1; skip[id]:
 * isBad() || IsInKeyFrame(pKF) when the loop reaches it.  best[k] out: the fused KF
 * keypoint or -1.  (Replace / AddObservation stay with the caller, in order.) */
void ora_fuse(const ora_frame* kf, const int32_t* points, int npoints, const uint8_t* skip, const ora_mappoints* mps,
              float th, int32_t* best) {
    ora_grid g;
    ora_grid_build(kf, &g);
    int* cand = (int*)malloc(sizeof(int) * (size_t)(kf->n + 1));
    float inv_sigma2[32];
    for (int l = 0; l < kf->nlevels; l++) inv_sigma2[l] = 1.0f / kf->level_sigma2[l];
    float Ow[3];
    for (int c = 0; c < 3; c++) Ow[c] = -(kf->Tcw[c] * kf->Tcw[3] + kf->Tcw[4 + c] * kf->Tcw[7] + kf->Tcw[8 + c] * kf->Tcw[11]);
    for (int k = 0; k < npoints; k++) {
        best[k] = -1;
        const int mp = points[k];
        if (mp < 0 || skip[mp]) continue;
        const float* p3Dw = mps->pos + 3 * (size_t)mp;
        float p3Dc[3];
        project(kf->Tcw, p3Dw, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
        const float u = mad_(kf->fx, x, kf->cx), v = mad_(kf->fy, y, kf->cy);
        if (!(u >= kf->min_x && u < kf->max_x && v >= kf->min_y && v < kf->max_y)) continue;
        const float ur = msub_(u, kf->bf, invz);
        const float maxDistance = 1.2f * mps->max_distance[mp], minDistance = 0.8f * mps->min_distance[mp];
        float PO[3];
        for (int c = 0; c < 3; c++) PO[c] = p3Dw[c] - Ow[c];
        const float dist3D = norm3(PO);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const float* Pn = mps->normal + 3 * (size_t)mp;
        double dot = 0.0;
        for (int c = 0; c < 3; c++) dot += (double)PO[c] * Pn[c];
        if (dot < 0.5 * dist3D) continue;
        const int pred = predict_scale(mps->max_distance[mp], dist3D, kf);
        const float radius = th * kf->scale_factors[pred];
        best[k] = window_best(kf, &g, cand, mps->desc + (size_t)mp * 32, u, v, ur, radius, pred, 1, inv_sigma2, TH_LOW);
    }
    free(cand);
    ora_grid_free(&g);
}

/* ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, th,
 * vector<MapPoint*>& vpReplacePoint), ORBmatcher.cc:1226-1352: the search part.
 * skip[id]: isBad() || in pKF->GetMapPoints(). */
void ora_fuse_sim3(const ora_frame* kf, const float* Scw, const int32_t* points, int npoints, const uint8_t* skip,
                   const ora_mappoints* mps, float th, int32_t* best) {
    ora_grid g;
    ora_grid_build(kf, &g);
    int* cand = (int*)malloc(sizeof(int) * (size_t)(kf->n + 1));
    double d0 = 0.0;
    for (int c = 0; c < 3; c++) d0 += (double)Scw[c] * Scw[c];
    const float scw = (float)sqrt(d0);
    const float alpha = (float)(1.0 / scw);
    float T[12];
    for (int k = 0; k < 12; k++) T[k] = Scw[k] * alpha;
    float Ow[3];
    for (int c = 0; c < 3; c++) Ow[c] = -(T[c] * T[3] + T[4 + c] * T[7] + T[8 + c] * T[11]);
    for (int k = 0; k < npoints; k++) {
        best[k] = -1;
        const int mp = points[k];
        if (mp < 0 || skip[mp]) continue;
        const float* p3Dw = mps->pos + 3 * (size_t)mp;
        float p3Dc[3];
        project(T, p3Dw, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = (float)(1.0 / p3Dc[2]);
        const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
        const float u = mad_(kf->fx, x, kf->cx), v = mad_(kf->fy, y, kf->cy);
        if (!(u >= kf->min_x && u < kf->max_x && v >= kf->min_y && v < kf->max_y)) continue;
        const float maxDistance = 1.2f * mps->max_distance[mp], minDistance = 0.8f * mps->min_distance[mp];
        float PO[3];
        for (int c = 0; c < 3; c++) PO[c] = p3Dw[c] - Ow[c];
        const float dist3D = norm3(PO);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const float* Pn = mps->normal + 3 * (size_t)mp;
        double dot = 0.0;
        for (int c = 0; c < 3; c++) dot += (double)PO[c] * Pn[c];
        if (dot < 0.5 * dist3D) continue;
        const int pred = predict_scale(mps->max_distance[mp], dist3D, kf);
        const float radius = th * kf->scale_factors[pred];
        best[k] = window_best(kf, &g, cand, mps->desc + (size_t)mp * 32, u, v, 0.f, radius, pred, 0, NULL, TH_LOW);
    }
    free(cand);
    ora_grid_free(&g);
}

/* One direction of SearchBySim3: MapPoints of `src` (ids src_mp, -1 = NULL) mapped
 * into `dst` by x_dst = sR * (R_src x + t_src) + t, window-searched in dst. */
static void sim3_direction(const ora_frame* src, const int32_t* src_mp, const uint8_t* already, const ora_frame* dst,
                           const ora_mappoints* mps, const float* sR, const float* t, float th, int* vnMatch) {
    ora_grid g;
    ora_grid_build(dst, &g);
    int* cand = (int*)malloc(sizeof(int) * (size_t)(dst->n + 1));
    for (int i = 0; i < src->n; i++) {
        vnMatch[i] = -1;
        const int mp = src_mp[i];
        if (mp < 0 || already[i]) continue;
        if (mps->bad && mps->bad[mp]) continue;
        const float* p3Dw = mps->pos + 3 * (size_t)mp;
        float pc[3], pd[3];
        project(src->Tcw, p3Dw, pc);
        for (int r = 0; r < 3; r++) pd[r] = sR[3 * r] * pc[0] + sR[3 * r + 1] * pc[1] + sR[3 * r + 2] * pc[2] + t[r];
        if (pd[2] < 0.0) continue;
        const float invz = (float)(1.0 / pd[2]);
        const float x = pd[0] * invz, y = pd[1] * invz;
        const float u = mad_(dst->fx, x, dst->cx), v = mad_(dst->fy, y, dst->cy);
        if (!(u >= dst->min_x && u < dst->max_x && v >= dst->min_y && v < dst->max_y)) continue;
        const float maxDistance = 1.2f * mps->max_distance[mp], minDistance = 0.8f * mps->min_distance[mp];
        const float dist3D = norm3(pd);
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int pred = predict_scale(mps->max_distance[mp], dist3D, dst);
        const float radius = th * dst->scale_factors[pred];
        vnMatch[i] = window_best(dst, &g, cand, mps->desc + (size_t)mp * 32, u, v, 0.f, radius, pred, 0, NULL, TH_HIGH);
    }
    free(cand);
    ora_grid_free(&g);
}

/* ORBmatcher::SearchBySim3, ORBmatcher.cc:1361-1602.  kf*_mp: GetMapPointMatches() as
 * ids; already1/2: vbAlreadyMatched1/2 (from the incoming vpMatches12); matches12 in/out
 * (KF2 MapPoint ids).  sR12 = s12*R12; sR21 = R12^T * (float)(1/s12); t21 = -sR21*t12.
 * Returns nFound. */
int ora_search_by_sim3(const ora_frame* kf1, const int32_t* mp1, const uint8_t* already1, const ora_frame* kf2,
                       const int32_t* mp2, const uint8_t* already2, const ora_mappoints* mps, float s12,
                       const float* R12, const float* t12, float th, int32_t* matches12) {
    float sR12[9], sR21[9], t21[3];
    const float inv = (float)(1.0 / s12);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            sR12[3 * r + c] = s12 * R12[3 * r + c];
            sR21[3 * r + c] = R12[3 * c + r] * inv;
        }
    for (int r = 0; r < 3; r++) t21[r] = -(sR21[3 * r] * t12[0] + sR21[3 * r + 1] * t12[1] + sR21[3 * r + 2] * t12[2]);
    int* vnMatch1 = (int*)malloc(sizeof(int) * (size_t)(kf1->n + 1));
    int* vnMatch2 = (int*)malloc(sizeof(int) * (size_t)(kf2->n + 1));
    sim3_direction(kf1, mp1, already1, kf2, mps, sR21, t21, th, vnMatch1);
    sim3_direction(kf2, mp2, already2, kf1, mps, sR12, t12, th, vnMatch2);
    int nFound = 0;
    for (int i1 = 0; i1 < kf1->n; i1++) {
        const int idx2 = vnMatch1[i1];
        if (idx2 >= 0 && vnMatch2[idx2] == i1) {
            matches12[i1] = mp2[idx2];
            nFound++;
        }
    }
    free(vnMatch1);
    free(vnMatch2);
    return nFound;
}

/* MapPoint::ComputeDistinctiveDescriptors, MapPoint.cc:295-360: descriptors of the
 * good observations in observation-map order; the one with the smallest median
 * distance (vDists[0.5*(N-1)], first on ties).  best[m] = index in the MapPoint's list
 * or -1 when it has none. */
void ora_distinctive_descriptors(int nmp, const int32_t* off, const uint8_t* desc, int32_t* best) {
    for (int m = 0; m < nmp; m++) {
        const int N = off[m + 1] - off[m];
        best[m] = -1;
        if (N <= 0) continue;
        const uint8_t* D = desc + (size_t)off[m] * 32;
        int* row = (int*)malloc(sizeof(int) * (size_t)N);
        int BestMedian = 0x7fffffff, BestIdx = 0;
        for (int i = 0; i < N; i++) {
            for (int j = 0; j < N; j++) row[j] = i == j ? 0 : hamming(D + (size_t)i * 32, D + (size_t)j * 32);
            for (int a = 1; a < N; a++) { /* insertion sort */
                const int x = row[a];
                int b = a - 1;
                while (b >= 0 && row[b] > x) {
                    row[b + 1] = row[b];
                    b--;
                }
                row[b + 1] = x;
            }
            const int median = row[(size_t)(0.5 * (N - 1))];
            if (median < BestMedian) {
                BestMedian = median;
                BestIdx = i;
            }
        }
        best[m] = BestIdx;
        free(row);
    }
}

/* ---------------------------------------------------------------- RGB-D Frame */

/* Frame::ComputeStereoFromRGBD (Frame.cc:888-909) on the image Tracking::GrabImageRGBD
 * hands the Frame (Tracking.cc:265-271): imDepth.convertTo(imDepth, CV_32F,
 * mDepthMapFactor) whenever |mDepthMapFactor - 1| > 1e-5 or the image is not CV_32F.
 * OpenCV 3.3.1's cvtScale16u32f / cvtScale32f compute in float: (float)src * (float)alpha
 * + (float)beta with beta = 0 (recalled, unpinned; the + 0 is exact either way).  Then for
 * keypoint i: d = imDepth.at<float>(v, u) with v = kp.pt.y, u = kp.pt.x of the distorted
 * keypoint converted to int (truncation), and where d > 0: mvDepth[i] = d, mvuRight[i] =
 * kpU.pt.x - mbf / d; otherwise both stay -1 (cc:889-890).  A keypoint outside the image
 * (never one the extractor produced) is given -1 here; the reference reads out of bounds. */
void ora_compute_stereo_from_rgbd(const ora_keypoint* keys, const ora_keypoint* keys_un, int n, const void* depth,
                                  int depth_f32, int width, int height, long long row_bytes, float depth_map_factor,
                                  float bf, float* u_right, float* out_depth) {
    const int convert = (fabsf(depth_map_factor - 1.0f) > 1e-5f) || !depth_f32;
    for (int i = 0; i < n; i++) {
        u_right[i] = -1.0f;
        out_depth[i] = -1.0f;
        const float v = keys[i].y, u = keys[i].x;
        const int iv = (int)v, iu = (int)u;
        if (iv < 0 || iv >= height || iu < 0 || iu >= width) continue;
        const unsigned char* row = (const unsigned char*)depth + (size_t)iv * (size_t)row_bytes;
        float d;
        if (depth_f32) {
            d = ((const float*)row)[iu];
            if (convert) d = d * depth_map_factor;
        } else {
            d = (float)((const uint16_t*)row)[iu] * depth_map_factor;
        }
        if (d > 0) {
            out_depth[i] = d;
            u_right[i] = keys_un[i].x - bf / d;
        }
    }
}

/* Tracking::TrackWithMotionModel's search (Tracking.cc:975-994): mvpMapPoints emptied,
 * SearchByProjection(CurrentFrame, LastFrame, th, bMono); with fewer than 20 matches,
 * emptied again and searched at 2*th.  *retried (optional) reports the second search. */
int ora_track_motion_model(const ora_frame* cur, int32_t* cur_mp, const ora_frame* last, const int32_t* last_mp,
                           const uint8_t* last_outlier, const ora_mappoints* mps, float th, int bMono, int check_ori,
                           int* retried) {
    for (int i = 0; i < cur->n; i++) cur_mp[i] = -1;
    int nm = ora_sbp_frame(cur, cur_mp, last, last_mp, last_outlier, mps, th, bMono, check_ori);
    if (retried) *retried = 0;
    if (nm < 20) {
        for (int i = 0; i < cur->n; i++) cur_mp[i] = -1;
        nm = ora_sbp_frame(cur, cur_mp, last, last_mp, last_outlier, mps, 2 * th, bMono, check_ori);
        if (retried) *retried = 1;
    }
    return nm;
}
