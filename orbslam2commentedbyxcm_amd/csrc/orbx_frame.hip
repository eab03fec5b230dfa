// orbx_frame.hip -- the per-frame steps between extraction and matching on the device
// (SURVEY.md §8(f) rank 3):
//   Frame::UndistortKeyPoints   Frame.cc:586-628  (cv::undistortPoints, OpenCV 3.3.1)
//   Frame::ComputeImageBounds   Frame.cc:636-665
//   Frame::AssignFeaturesToGrid Frame.cc:351-370  (+ PosInGrid 558-567)
//   the stereo / RGB-D MapPoints of a new keyframe (Tracking.cc:1069-1121):
//   Frame::UnprojectStereo Frame.cc:912-927 + MapPoint::UpdateNormalAndDepth MapPoint.cc:386-439
// so a batch extracted by orbx_extract_batch_device gets mvKeysUn and mGrid without a
// host round trip.  Undistortion is one thread per keypoint in double precision (the
// 5-iteration fixed point of cvUndistortPoints, same operation order as the oracle,
// no contraction).  The grid is one 1024-thread workgroup per frame: keys
// (cell << 32 | index) are block-sorted (orbx_block_sort.h), so each cell's list is in
// ascending index order like the reference's push_back loop, and written as CSR.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "orbx.h"
#include "orbx_block_sort.h"
#include "orbx_error.h"
#include "orbx_match_types.h"

using namespace orbx;

namespace orbx {

struct CamDev {
    double fx, fy, cx, cy, ifx, ify;
    double k[5];
    int enabled;  // mDistCoef.at<float>(0) != 0
};

// cvUndistortPoints for one point (see oracle/orbx_oracle_match.c ora_undistort_points)
__device__ __forceinline__ void undistort_point(const CamDev& C, float u, float v, float& ou, float& ov) {
    double x = u, y = v;
    x = __dmul_rn(__dsub_rn(x, C.cx), C.ifx);
    y = __dmul_rn(__dsub_rn(y, C.cy), C.ify);
    const double x0 = x, y0 = y;
    const double* k = C.k;
    for (int j = 0; j < 5; j++) {
        const double r2 = __dadd_rn(__dmul_rn(x, x), __dmul_rn(y, y));
        // (1 + ((k7*r2 + k6)*r2 + k5)*r2) with k5..k7 = 0 is exactly 1
        const double num = __dadd_rn(1.0, __dmul_rn(__dadd_rn(__dmul_rn(__dadd_rn(__dmul_rn(0.0, r2), 0.0), r2), 0.0), r2));
        const double den = __dadd_rn(1.0, __dmul_rn(__dadd_rn(__dmul_rn(__dadd_rn(__dmul_rn(k[4], r2), k[1]), r2), k[0]), r2));
        const double icdist = num / den;
        // 2*k2*x*y + k3*(r2 + 2*x*x) + k8*r2 + k9*r2*r2
        const double dX = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(__dmul_rn(__dmul_rn(2.0, k[2]), x), y),
                                                        __dmul_rn(k[3], __dadd_rn(r2, __dmul_rn(__dmul_rn(2.0, x), x)))),
                                              __dmul_rn(0.0, r2)),
                                    __dmul_rn(__dmul_rn(0.0, r2), r2));
        // k2*(r2 + 2*y*y) + 2*k3*x*y + k10*r2 + k11*r2*r2
        const double dY = __dadd_rn(__dadd_rn(__dadd_rn(__dmul_rn(k[2], __dadd_rn(r2, __dmul_rn(__dmul_rn(2.0, y), y))),
                                                        __dmul_rn(__dmul_rn(__dmul_rn(2.0, k[3]), x), y)),
                                              __dmul_rn(0.0, r2)),
                                    __dmul_rn(__dmul_rn(0.0, r2), r2));
        x = __dmul_rn(__dsub_rn(x0, dX), icdist);
        y = __dmul_rn(__dsub_rn(y0, dY), icdist);
    }
    const double xx = __dadd_rn(__dadd_rn(__dmul_rn(C.fx, x), __dmul_rn(0.0, y)), C.cx);
    const double yy = __dadd_rn(__dadd_rn(__dmul_rn(0.0, x), __dmul_rn(C.fy, y)), C.cy);
    const double ww = 1.0 / __dadd_rn(__dadd_rn(__dmul_rn(0.0, x), __dmul_rn(0.0, y)), 1.0);
    ou = (float)__dmul_rn(xx, ww);
    ov = (float)__dmul_rn(yy, ww);
}

__global__ __launch_bounds__(256) void k_undistort(CamDev C, const orbx_keypoint* __restrict__ kin,
                                                   const int32_t* __restrict__ nper, int cap,
                                                   orbx_keypoint* __restrict__ kout) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n = min(nper[b], cap);
    if (i >= n) return;
    const size_t s = (size_t)b * cap + i;
    orbx_keypoint kp = kin[s];
    if (C.enabled) undistort_point(C, kp.x, kp.y, kp.x, kp.y);
    kout[s] = kp;
}

// The RGB-D Frame's steps after ExtractORB (Frame.cc:227-230), one thread per keypoint
// slot: UndistortKeyPoints (UNDIST; else mvKeysUn is read) and ComputeStereoFromRGBD
// (Frame.cc:888-909) with GrabImageRGBD's convertTo(CV_32F, mDepthMapFactor)
// (Tracking.cc:265-271) applied to the one pixel each keypoint reads -- the conversion is
// per pixel, so converting only what is read gives the same floats without a pass over
// the image.  OpenCV 3.3.1's cvtScale to 32F computes in float: d = (float)src * scale
// (+ 0, exact).  The lookup index is imDepth.at<float>(v, u) of the distorted keypoint:
// float -> int conversions, i.e. truncation (the coordinates are >= 0).
struct RgbdArgs {
    const orbx_keypoint* kps;
    orbx_keypoint* kps_un;
    const int32_t* n;
    int cap;
    const unsigned char* depth;
    long long row_bytes, frame_bytes;
    int width, height;
    int f32;        // depth image of floats (else u16)
    int scale;      // apply `factor` (u16: always; f32: when |factor - 1| > 1e-5)
    float factor;   // mDepthMapFactor
    float bf;
    float* u_right;
    float* depth_out;
};

template <bool UNDIST>
__global__ __launch_bounds__(256) void k_rgbd_frame(CamDev C, RgbdArgs A) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= A.cap) return;
    const int n = min(A.n[b], A.cap);
    const size_t s = (size_t)b * A.cap + i;
    float ur = -1.f, dd = -1.f;
    if (i < n) {
        const orbx_keypoint kp = A.kps[s];
        orbx_keypoint kpu;
        if constexpr (UNDIST) {
            kpu = kp;
            if (C.enabled) undistort_point(C, kp.x, kp.y, kpu.x, kpu.y);
            A.kps_un[s] = kpu;
        } else {
            kpu = A.kps_un[s];
        }
        const int v = (int)kp.y, u = (int)kp.x;  // Mat::at<float>(int, int) of float arguments
        if (v >= 0 && v < A.height && u >= 0 && u < A.width) {
            const unsigned char* row = A.depth + (size_t)b * A.frame_bytes + (size_t)v * A.row_bytes;
            float d;
            if (A.f32) {
                d = ((const float*)row)[u];
                if (A.scale) d = __fmul_rn(d, A.factor);
            } else {
                d = __fmul_rn((float)((const uint16_t*)row)[u], A.factor);
            }
            if (d > 0) {
                dd = d;
                ur = __fsub_rn(kpu.x, __fdiv_rn(A.bf, d));  // kpU.pt.x - mbf / d
            }
        }
    }
    A.u_right[s] = ur;
    A.depth_out[s] = dd;
}

// Image corners for ComputeImageBounds (4 points)
__global__ void k_undistort_points(CamDev C, const float* __restrict__ pts, int n, float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) undistort_point(C, pts[2 * i], pts[2 * i + 1], out[2 * i], out[2 * i + 1]);
}

struct GridArgs {
    float min_x, min_y, inv_w, inv_h;
};

// Frame::AssignFeaturesToGrid for frame blockIdx.x: cell_start [kGridCols*kGridRows + 1],
// cell_idx [cap] (the first cell_start[last] entries are valid).
__global__ __launch_bounds__(kSortThreads) void k_grid(GridArgs G, const orbx_keypoint* __restrict__ keys,
                                                       const int32_t* __restrict__ nper, int cap,
                                                       int32_t* __restrict__ cell_start, int32_t* __restrict__ cell_idx) {
    extern __shared__ unsigned long long s_key[];
    constexpr int kCells = kGridCols * kGridRows;
    const int b = blockIdx.x;
    const int n = min(nper[b], cap);
    int ne = 1;
    while (ne * kSortThreads < n) ne <<= 1;
    const int m = ne * kSortThreads;
    unsigned long long r[kSortPer];
#pragma unroll
    for (int e = 0; e < kSortPer; e++) {
        const int i = e * kSortThreads + threadIdx.x;
        unsigned long long key = ~0ull;
        if (e < ne && i < n) {
            const orbx_keypoint kp = keys[(size_t)b * cap + i];
            const int px = (int)roundf(__fmul_rn(__fsub_rn(kp.x, G.min_x), G.inv_w));  // PosInGrid
            const int py = (int)roundf(__fmul_rn(__fsub_rn(kp.y, G.min_y), G.inv_h));
            if (!(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows))
                key = (unsigned long long)(unsigned)(px * kGridRows + py) << 32 | (unsigned)i;
        }
        r[e] = key;
    }
    block_bitonic_sort64(r, ne, s_key);
    int32_t* cs = cell_start + (size_t)b * (kCells + 1);
    int32_t* ci = cell_idx + (size_t)b * cap;
    // cell_start[c] = first sorted position with cell >= c
    for (int p = threadIdx.x; p < m; p += kSortThreads) {
        const unsigned long long k = s_key[p];
        const int c = k == ~0ull ? kCells : (int)(k >> 32);
        const int cprev = p == 0 ? -1 : (s_key[p - 1] == ~0ull ? kCells : (int)(s_key[p - 1] >> 32));
        for (int q = cprev + 1; q <= c; q++) cs[q] = p;
        if (c < kCells) ci[p] = (int32_t)(unsigned)k;
        if (p == m - 1)
            for (int q = c + 1; q <= kCells; q++) cs[q] = m;  // every key valid: tail cells start at m
    }
}

// Tracking::CreateNewKeyFrame's MapPoints of B frames (one thread per keypoint slot, id
// b*cap + i): Frame::UnprojectStereo (x3Dc = ((u-cx)*z*invfx, (v-cy)*z*invfy, z), Pos =
// Rwc*x3Dc + Ow) and UpdateNormalAndDepth with the frame as the only observation (normal =
// PC * (float)(1/|PC|), mfMaxDistance = |PC| * mvScaleFactors[octave], mfMinDistance =
// mfMaxDistance / mvScaleFactors[nLevels-1]).  Float products summed left to right, norms
// in double.  Slots without a keypoint or with z <= 0: bad.
struct MapPointArgs {
    const orbx_keypoint* kps;
    const int32_t* n;
    int cap;
    const float* depth;    // [B][cap] mvDepth or null (const_depth for every keypoint)
    float const_depth;
    const float* Tcw;      // [B][12]
    float fx, fy, cx, cy;
    float scale[32];
    int nlevels;
    float* pos;
    float* normal;
    float* max_distance;
    float* min_distance;
    int32_t* observations;
    uint8_t* bad;
};

__global__ __launch_bounds__(256) void k_create_mappoints(MapPointArgs A, int total) {
    const int id = blockIdx.x * 256 + threadIdx.x;
    if (id >= total) return;
    const int b = id / A.cap, i = id - b * A.cap;
    const int n = A.n[b] < A.cap ? A.n[b] : A.cap;
    const float z = i < n ? (A.depth ? A.depth[id] : A.const_depth) : 0.f;
    A.observations[id] = 0;
    A.bad[id] = 1;
    if (!(z > 0)) return;  // UnprojectStereo returns an empty Mat
    const orbx_keypoint kp = A.kps[id];
    const float* T = A.Tcw + 12 * (size_t)b;
    const float invfx = 1.0f / A.fx, invfy = 1.0f / A.fy;
    const float x = (kp.x - A.cx) * z * invfx;
    const float y = (kp.y - A.cy) * z * invfy;
    float Ow[3], P[3], PC[3];
    for (int r = 0; r < 3; r++) Ow[r] = -(T[r] * T[3] + T[4 + r] * T[7] + T[8 + r] * T[11]);
    for (int r = 0; r < 3; r++) P[r] = T[r] * x + T[4 + r] * y + T[8 + r] * z + Ow[r];  // Rwc[r][c] = Rcw[c][r]
    double ss = 0.0;
    for (int c = 0; c < 3; c++) {
        PC[c] = P[c] - Ow[c];
        ss += (double)PC[c] * (double)PC[c];
    }
    const double nrm = sqrt(ss);
    const float inv = (float)(1.0 / nrm);
    const float dist = (float)nrm;
    const int oct = kp.octave < 0 ? 0 : (kp.octave >= A.nlevels ? A.nlevels - 1 : kp.octave);
    const float mx = dist * A.scale[oct];
    for (int c = 0; c < 3; c++) {
        A.pos[3 * (size_t)id + c] = P[c];
        A.normal[3 * (size_t)id + c] = PC[c] * inv;
    }
    A.max_distance[id] = mx;
    A.min_distance[id] = mx / A.scale[A.nlevels - 1];
    A.observations[id] = 1;
    A.bad[id] = 0;
}

// Tracking::UpdateLastFrame (Tracking.cc:893-954) for B stereo LastFrames, one 256-thread
// workgroup per frame.  The reference sorts (mvDepth[i], i) for depth > 0 and visits the
// pairs in order, giving a keypoint without a MapPoint (or with Observations() < 1) a
// temporal MapPoint at UnprojectStereo(i), until it has visited more than 100 points and the
// current one lies beyond mThDepth.  With c points at depth <= th_depth among m with depth,
// the visited set is therefore the K = min(m, max(c, 100) + 1) smallest (depth, index)
// pairs: every point within th_depth, plus the nearest kb = K - c beyond it -- one (the
// minimum key) when c >= 100, and otherwise ranked by counting.  No sort is needed.
// Keys (float bits of depth << 32 | index) order like the pairs: depths are positive.
struct LastFrameArgs {
    const orbx_keypoint* kps;
    const int32_t* n;
    int cap;
    const float* depth;      // [B][cap] mvDepth
    const float* Tcw;        // [B][12]
    float fx, fy, cx, cy;
    float th_depth;          // mThDepth
    const int32_t* obs_in;   // [B][cap] Observations() of LastFrame's MapPoints (-1 = NULL) or null
    const float* pos_in;     // [B][cap][3] their GetWorldPos() (read where obs_in >= 0)
    int32_t* mp_obs;         // [B][cap] out (-1 = no MapPoint; 0 = temporal)
    float* mp_pos;           // [B][cap][3] out
    uint8_t* has_mp;         // [B][cap] out
};

constexpr int kLastFrameThreads = 256;

__global__ __launch_bounds__(kLastFrameThreads) void k_update_last_frame(LastFrameArgs A) {
    const int b = blockIdx.x;
    const int t = threadIdx.x;
    const int n = A.n[b] < A.cap ? A.n[b] : A.cap;
    const size_t base = (size_t)b * A.cap;
    const float* dep = A.depth + base;
    __shared__ int s_c, s_m;
    __shared__ unsigned long long s_min;
    if (t == 0) {
        s_c = 0;
        s_m = 0;
        s_min = ~0ull;
    }
    __syncthreads();
    int c = 0, m = 0;
    unsigned long long mn = ~0ull;
    for (int i = t; i < n; i += kLastFrameThreads) {
        const float z = dep[i];
        if (z > 0) {
            m++;
            if (z <= A.th_depth) {
                c++;
            } else {
                const unsigned long long k = (unsigned long long)__float_as_uint(z) << 32 | (unsigned)i;
                mn = k < mn ? k : mn;
            }
        }
    }
    if (c) atomicAdd(&s_c, c);
    if (m) atomicAdd(&s_m, m);
    if (mn != ~0ull) atomicMin(&s_min, mn);
    __syncthreads();
    const int C = s_c, M = s_m;
    const int K = M < (C > 100 ? C : 100) + 1 ? M : (C > 100 ? C : 100) + 1;
    const int kb = K - C;  // beyond-threshold points visited
    const float* T = A.Tcw + 12 * (size_t)b;
    const float invfx = 1.0f / A.fx, invfy = 1.0f / A.fy;
    float Ow[3];
    for (int r = 0; r < 3; r++) Ow[r] = -(T[r] * T[3] + T[4 + r] * T[7] + T[8 + r] * T[11]);
    for (int i = t; i < A.cap; i += kLastFrameThreads) {
        int obs = -1;
        float p[3] = {0.f, 0.f, 0.f};
        if (i < n) {
            if (A.obs_in) {
                obs = A.obs_in[base + i];
                if (obs >= 0)
                    for (int r = 0; r < 3; r++) p[r] = A.pos_in[3 * (base + i) + r];
            }
            const float z = dep[i];
            bool visited = false;
            if (z > 0) {
                if (z <= A.th_depth) {
                    visited = true;
                } else if (kb > 0) {
                    const unsigned long long k = (unsigned long long)__float_as_uint(z) << 32 | (unsigned)i;
                    if (kb == 1) {
                        visited = k == s_min;
                    } else {  // c < 100: rank among the beyond-threshold keys (rare)
                        int rank = 0;
                        for (int j = 0; j < n && rank < kb; j++) {
                            const float zj = dep[j];
                            if (zj > 0 && zj > A.th_depth)  // the pairs with depth only (cc:909-913)
                                rank += ((unsigned long long)__float_as_uint(zj) << 32 | (unsigned)j) < k;
                        }
                        visited = rank < kb;
                    }
                }
            }
            if (visited && obs < 1) {  // !pMP || pMP->Observations() < 1: new temporal MapPoint
                const orbx_keypoint kp = A.kps[base + i];
                const float x = (kp.x - A.cx) * z * invfx;
                const float y = (kp.y - A.cy) * z * invfy;
                for (int r = 0; r < 3; r++) p[r] = T[r] * x + T[4 + r] * y + T[8 + r] * z + Ow[r];
                obs = 0;
            }
        }
        A.mp_obs[base + i] = obs;
        A.has_mp[base + i] = obs >= 0;
        for (int r = 0; r < 3; r++) A.mp_pos[3 * (base + i) + r] = p[r];
    }
}

}  // namespace orbx

namespace {

int fail(int code, const char* what) {
    set_last_error(what);
    return code;
}

#define HIP_TRY(expr)                                                               \
    do {                                                                            \
        hipError_t _e = (expr);                                                     \
        if (_e != hipSuccess) {                                                     \
            set_last_error(std::string(#expr) + ": " + hipGetErrorString(_e));      \
            return ORBX_ERR_HIP;                                                    \
        }                                                                           \
    } while (0)

CamDev cam_dev(const orbx_camera* c) {
    CamDev C;
    C.fx = c->fx;
    C.fy = c->fy;
    C.cx = c->cx;
    C.cy = c->cy;
    C.ifx = 1.0 / C.fx;
    C.ify = 1.0 / C.fy;
    C.k[0] = c->k1;
    C.k[1] = c->k2;
    C.k[2] = c->p1;
    C.k[3] = c->p2;
    C.k[4] = c->k3;
    C.enabled = c->k1 != 0.0f;
    return C;
}

bool bounds_ok(const float* bd) { return bd && bd[1] > bd[0] && bd[3] > bd[2]; }

GridArgs grid_args(const float* bd) {
    GridArgs G;
    G.min_x = bd[0];
    G.min_y = bd[2];
    G.inv_w = (float)kGridCols / (bd[1] - bd[0]);  // Frame.cc:157-159
    G.inv_h = (float)kGridRows / (bd[3] - bd[2]);
    return G;
}

hipError_t launch_grid(const GridArgs& G, int batch, const orbx_keypoint* keys, const int32_t* n, int cap,
                       int32_t* cell_start, int32_t* cell_idx, hipStream_t s) {
    int np = kSortThreads;
    while (np < cap) np <<= 1;
    const size_t lds = (size_t)np * 8;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)k_grid, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_grid, dim3(batch), dim3(kSortThreads), lds, s, G, keys, n, cap, cell_start, cell_idx);
    return hipGetLastError();
}

}  // namespace

extern "C" {

int orbx_undistort_keypoints_device(const orbx_camera* cam, int batch, const orbx_keypoint* d_keys, const int32_t* d_n,
                                    int cap, orbx_keypoint* d_keys_un, void* stream) {
    if (!cam || batch < 0 || cap < 0 || (batch && cap && (!d_keys || !d_n || !d_keys_un)))
        return fail(ORBX_ERR_ARG, "bad argument");
    if (!batch || !cap) return ORBX_OK;
    const dim3 g((cap + 255) / 256, batch);
    hipLaunchKernelGGL(k_undistort, g, dim3(256), 0, (hipStream_t)stream, cam_dev(cam), d_keys, d_n, cap, d_keys_un);
    HIP_TRY(hipGetLastError());
    return ORBX_OK;
}

int orbx_undistort_keypoints(int device, const orbx_camera* cam, const orbx_keypoint* keys, int n,
                             orbx_keypoint* keys_un) {
    if (!cam || n < 0 || (n && (!keys || !keys_un))) return fail(ORBX_ERR_ARG, "bad argument");
    if (n == 0) return ORBX_OK;
    if (cam->k1 == 0.0f) {  // mvKeysUn = mvKeys (Frame.cc:587-590)
        if (keys_un != keys) std::memcpy(keys_un, keys, sizeof(orbx_keypoint) * (size_t)n);
        return ORBX_OK;
    }
    HIP_TRY(hipSetDevice(device));
    orbx_keypoint* d = nullptr;
    int32_t* d_n = nullptr;
    HIP_TRY(hipMalloc((void**)&d, sizeof(orbx_keypoint) * (size_t)n * 2));
    hipError_t e = hipMalloc((void**)&d_n, sizeof(int32_t));
    if (e == hipSuccess) e = hipMemcpy(d, keys, sizeof(orbx_keypoint) * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_n, &n, sizeof(int32_t), hipMemcpyHostToDevice);
    int rc = ORBX_OK;
    if (e == hipSuccess) rc = orbx_undistort_keypoints_device(cam, 1, d, d_n, n, d + n, nullptr);
    if (e == hipSuccess && rc == ORBX_OK)
        e = hipMemcpy(keys_un, d + n, sizeof(orbx_keypoint) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (d_n) (void)hipFree(d_n);
    if (rc != ORBX_OK) return rc;
    HIP_TRY(e);
    return ORBX_OK;
}

int orbx_compute_image_bounds(int device, const orbx_camera* cam, int cols, int rows, float* bounds) {
    if (!cam || !bounds || cols <= 0 || rows <= 0) return fail(ORBX_ERR_ARG, "bad argument");
    if (cam->k1 == 0.0f) {
        bounds[0] = 0.0f;
        bounds[1] = (float)cols;
        bounds[2] = 0.0f;
        bounds[3] = (float)rows;
        return ORBX_OK;
    }
    const float c[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
    float u[8];
    HIP_TRY(hipSetDevice(device));
    float* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, sizeof(c) * 2));
    hipError_t e = hipMemcpy(d, c, sizeof(c), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_undistort_points, dim3(1), dim3(64), 0, nullptr, cam_dev(cam), d, 4, d + 8);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(u, d + 8, sizeof(u), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    HIP_TRY(e);
    bounds[0] = u[0] < u[4] ? u[0] : u[4];  // min(top-left x, bottom-left x)
    bounds[1] = u[2] > u[6] ? u[2] : u[6];  // max(top-right x, bottom-right x)
    bounds[2] = u[1] < u[3] ? u[1] : u[3];  // min(top-left y, top-right y)
    bounds[3] = u[5] > u[7] ? u[5] : u[7];  // max(bottom-left y, bottom-right y)
    return ORBX_OK;
}

int orbx_create_mappoints_device(int batch, const orbx_keypoint* d_kps, const int32_t* d_n, int cap,
                                 const float* d_depth, float const_depth, const float* d_Tcw, float fx, float fy,
                                 float cx, float cy, const float* scale_factors, int nlevels, float* d_pos,
                                 float* d_normal, float* d_max_distance, float* d_min_distance,
                                 int32_t* d_observations, uint8_t* d_bad, void* stream) {
    if (batch < 0 || cap <= 0 || !scale_factors || nlevels < 1 || nlevels > 32) return fail(ORBX_ERR_ARG, "bad argument");
    if (batch == 0) return ORBX_OK;
    if (!d_kps || !d_n || !d_Tcw || !d_pos || !d_normal || !d_max_distance || !d_min_distance || !d_observations ||
        !d_bad)
        return fail(ORBX_ERR_ARG, "null buffer");
    MapPointArgs A{};
    A.kps = d_kps;
    A.n = d_n;
    A.cap = cap;
    A.depth = d_depth;
    A.const_depth = const_depth;
    A.Tcw = d_Tcw;
    A.fx = fx;
    A.fy = fy;
    A.cx = cx;
    A.cy = cy;
    for (int l = 0; l < nlevels; l++) A.scale[l] = scale_factors[l];
    A.nlevels = nlevels;
    A.pos = d_pos;
    A.normal = d_normal;
    A.max_distance = d_max_distance;
    A.min_distance = d_min_distance;
    A.observations = d_observations;
    A.bad = d_bad;
    const long long total = (long long)batch * cap;
    if (total >= (1ll << 31)) return fail(ORBX_ERR_ARG, "batch * cap too large");
    hipLaunchKernelGGL(k_create_mappoints, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, A,
                       (int)total);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ORBX_ERR_HIP, hipGetErrorString(e));
    return ORBX_OK;
}

int orbx_update_last_frame_device(int batch, const orbx_keypoint* d_kps, const int32_t* d_n, int cap,
                                  const float* d_depth, const float* d_Tcw, float fx, float fy, float cx, float cy,
                                  float th_depth, const int32_t* d_obs_in, const float* d_pos_in, int32_t* d_mp_obs,
                                  float* d_mp_pos, uint8_t* d_has_mp, void* stream) {
    if (batch < 0 || cap <= 0) return fail(ORBX_ERR_ARG, "bad argument");
    if (batch == 0) return ORBX_OK;
    if (!d_kps || !d_n || !d_depth || !d_Tcw || !d_mp_obs || !d_mp_pos || !d_has_mp || (d_obs_in && !d_pos_in))
        return fail(ORBX_ERR_ARG, "null buffer");
    if (!(fx != 0.f) || !(fy != 0.f)) return fail(ORBX_ERR_ARG, "fx, fy must be non-zero");
    LastFrameArgs A{};
    A.kps = d_kps;
    A.n = d_n;
    A.cap = cap;
    A.depth = d_depth;
    A.Tcw = d_Tcw;
    A.fx = fx;
    A.fy = fy;
    A.cx = cx;
    A.cy = cy;
    A.th_depth = th_depth;
    A.obs_in = d_obs_in;
    A.pos_in = d_pos_in;
    A.mp_obs = d_mp_obs;
    A.mp_pos = d_mp_pos;
    A.has_mp = d_has_mp;
    hipLaunchKernelGGL(k_update_last_frame, dim3(batch), dim3(kLastFrameThreads), 0, (hipStream_t)stream, A);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(ORBX_ERR_HIP, hipGetErrorString(e));
    return ORBX_OK;
}

int orbx_compute_stereo_from_rgbd_device(const orbx_camera* cam, const orbx_rgbd_batch* rb, void* stream) {
    if (!rb || rb->batch < 0 || rb->cap < 0) return fail(ORBX_ERR_ARG, "bad argument");
    if (!rb->batch || !rb->cap) return ORBX_OK;
    if (!rb->kps || !rb->kps_un || !rb->n || !rb->depth || !rb->u_right || !rb->depth_out)
        return fail(ORBX_ERR_ARG, "null buffer");
    if (rb->depth_type != ORBX_DEPTH_U16 && rb->depth_type != ORBX_DEPTH_F32)
        return fail(ORBX_ERR_ARG, "depth_type must be ORBX_DEPTH_U16 or ORBX_DEPTH_F32");
    const long long px = rb->depth_type == ORBX_DEPTH_U16 ? 2 : 4;
    if (rb->width <= 0 || rb->height <= 0 || rb->row_bytes < px * rb->width || rb->row_bytes % px ||
        (rb->batch > 1 && rb->frame_bytes < rb->row_bytes * rb->height) || rb->frame_bytes % px ||
        (uintptr_t)rb->depth % px)
        return fail(ORBX_ERR_ARG, "depth image geometry (sizes, row / frame strides, alignment)");
    RgbdArgs A{};
    A.kps = rb->kps;
    A.kps_un = rb->kps_un;
    A.n = rb->n;
    A.cap = rb->cap;
    A.depth = (const unsigned char*)rb->depth;
    A.row_bytes = rb->row_bytes;
    A.frame_bytes = rb->frame_bytes;
    A.width = rb->width;
    A.height = rb->height;
    A.f32 = rb->depth_type == ORBX_DEPTH_F32;
    // Tracking.cc:266: a CV_32F image is converted only when the factor is not ~1; the
    // conversion from 16U always runs (with alpha == 1 it is the plain conversion, equal
    // to a multiply by 1.0f)
    A.scale = !A.f32 || std::fabs(rb->depth_map_factor - 1.0f) > 1e-5;
    A.factor = rb->depth_map_factor;
    A.bf = rb->bf;
    A.u_right = rb->u_right;
    A.depth_out = rb->depth_out;
    const dim3 g((rb->cap + 255) / 256, rb->batch);
    if (cam) {
        hipLaunchKernelGGL(k_rgbd_frame<true>, g, dim3(256), 0, (hipStream_t)stream, cam_dev(cam), A);
    } else {
        hipLaunchKernelGGL(k_rgbd_frame<false>, g, dim3(256), 0, (hipStream_t)stream, CamDev{}, A);
    }
    HIP_TRY(hipGetLastError());
    return ORBX_OK;
}

int orbx_compute_stereo_from_rgbd(int device, const orbx_camera* cam, const orbx_keypoint* keys, int n,
                                  const void* depth, int depth_type, int width, int height, size_t row_bytes,
                                  float depth_map_factor, float bf, orbx_keypoint* keys_un, float* u_right,
                                  float* depth_out) {
    if (n < 0 || (n && (!keys || !keys_un || !u_right || !depth_out || !depth))) return fail(ORBX_ERR_ARG, "bad argument");
    if (n == 0) return ORBX_OK;  // Frame.cc:223-224: no keypoints, nothing computed
    if (depth_type != ORBX_DEPTH_U16 && depth_type != ORBX_DEPTH_F32) return fail(ORBX_ERR_ARG, "bad depth_type");
    const size_t px = depth_type == ORBX_DEPTH_U16 ? 2 : 4;
    if (width <= 0 || height <= 0 || row_bytes < px * (size_t)width) return fail(ORBX_ERR_ARG, "bad depth image");
    HIP_TRY(hipSetDevice(device));
    const size_t ib = px * (size_t)width * height, kb = sizeof(orbx_keypoint) * (size_t)n, fb = sizeof(float) * (size_t)n;
    char* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, ib + 2 * kb + 2 * fb + 256));
    orbx_keypoint* d_k = (orbx_keypoint*)d;
    orbx_keypoint* d_ku = d_k + n;
    float* d_ur = (float*)(d + 2 * kb);
    float* d_dp = d_ur + n;
    int32_t* d_n = (int32_t*)(d + 2 * kb + 2 * fb);
    void* d_img = d + 2 * kb + 2 * fb + 16;
    d_img = (void*)(((uintptr_t)d_img + 15) & ~(uintptr_t)15);
    hipError_t e = hipMemcpy2D(d_img, px * width, depth, row_bytes, px * width, height, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_k, keys, kb, hipMemcpyHostToDevice);
    if (e == hipSuccess && !cam) e = hipMemcpy(d_ku, keys_un, kb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_n, &n, sizeof(int32_t), hipMemcpyHostToDevice);
    int rc = ORBX_OK;
    if (e == hipSuccess) {
        orbx_rgbd_batch rb{};
        rb.batch = 1;
        rb.kps = d_k;
        rb.kps_un = d_ku;
        rb.n = d_n;
        rb.cap = n;
        rb.depth = d_img;
        rb.depth_type = depth_type;
        rb.width = width;
        rb.height = height;
        rb.row_bytes = (long long)(px * width);
        rb.frame_bytes = (long long)ib;
        rb.depth_map_factor = depth_map_factor;
        rb.bf = bf;
        rb.u_right = d_ur;
        rb.depth_out = d_dp;
        rc = orbx_compute_stereo_from_rgbd_device(cam, &rb, nullptr);
    }
    if (e == hipSuccess && rc == ORBX_OK && cam) e = hipMemcpy(keys_un, d_ku, kb, hipMemcpyDeviceToHost);
    if (e == hipSuccess && rc == ORBX_OK) e = hipMemcpy(u_right, d_ur, fb, hipMemcpyDeviceToHost);
    if (e == hipSuccess && rc == ORBX_OK) e = hipMemcpy(depth_out, d_dp, fb, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (rc != ORBX_OK) return rc;
    HIP_TRY(e);
    return ORBX_OK;
}

int orbx_assign_features_to_grid_device(int batch, const orbx_keypoint* d_keys_un, const int32_t* d_n, int cap,
                                        const float* bounds, int32_t* d_cell_start, int32_t* d_cell_idx,
                                        void* stream) {
    if (batch < 0 || cap < 0 || !bounds_ok(bounds) || (batch && (!d_keys_un || !d_n || !d_cell_start || !d_cell_idx)))
        return fail(ORBX_ERR_ARG, "bad argument");
    if (cap > kSortMaxKeys) return fail(ORBX_ERR_UNSUPPORTED, "more than 8192 keypoints per frame");
    if (!batch) return ORBX_OK;
    HIP_TRY(launch_grid(grid_args(bounds), batch, d_keys_un, d_n, cap < 1 ? 1 : cap, d_cell_start, d_cell_idx,
                        (hipStream_t)stream));
    return ORBX_OK;
}

int orbx_assign_features_to_grid(int device, const orbx_keypoint* keys_un, int n, const float* bounds,
                                 int32_t* cell_start, int32_t* cell_idx) {
    if (n < 0 || !bounds_ok(bounds) || !cell_start || (n && (!keys_un || !cell_idx)))
        return fail(ORBX_ERR_ARG, "bad argument");
    if (n > kSortMaxKeys) return fail(ORBX_ERR_UNSUPPORTED, "more than 8192 keypoints per frame");
    constexpr int kCells = kGridCols * kGridRows;
    if (n == 0) {
        for (int c = 0; c <= kCells; c++) cell_start[c] = 0;
        return ORBX_OK;
    }
    HIP_TRY(hipSetDevice(device));
    char* d = nullptr;
    const size_t bk = sizeof(orbx_keypoint) * (size_t)n, bs = sizeof(int32_t) * (kCells + 1),
                 bi = sizeof(int32_t) * (size_t)n;
    HIP_TRY(hipMalloc((void**)&d, bk + bs + bi + 256));
    orbx_keypoint* d_k = (orbx_keypoint*)d;
    int32_t* d_s = (int32_t*)(d + bk);
    int32_t* d_i = (int32_t*)(d + bk + bs);
    int32_t* d_n = (int32_t*)(d + bk + bs + bi);
    hipError_t e = hipMemcpy(d_k, keys_un, bk, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_n, &n, sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_grid(grid_args(bounds), 1, d_k, d_n, n, d_s, d_i, nullptr);
    if (e == hipSuccess) e = hipMemcpy(cell_start, d_s, bs, hipMemcpyDeviceToHost);
    if (e == hipSuccess && cell_start[kCells] > 0)
        e = hipMemcpy(cell_idx, d_i, sizeof(int32_t) * (size_t)cell_start[kCells], hipMemcpyDeviceToHost);
    (void)hipFree(d);
    HIP_TRY(e);
    return ORBX_OK;
}

}  // extern "C"
