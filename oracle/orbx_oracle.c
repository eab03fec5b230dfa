/*
 * orbx_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU parity checker.
 *
 * Plain-C restatement of ORB-SLAM2's ORBextractor::operator() and
 * ORBmatcher::DescriptorDistance.  Every function cites the reference file:line it
 * restates (paths relative to /root/reference).  Loaded only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product.
 *
 * Parity status: "parity unpinned" against the reference binary -- see
 * orbx_oracle.h and DESIGN.md §Parity.  OpenCV 3.3.1 internals are restated from
 * OpenCV's published algorithm (resize INTER_LINEAR fixed point, GaussianBlur
 * 8U fixed point, FAST_t<16>, fastAtan2, cvRound), scalar x86 semantics.
 *
 * Build: gcc -O2 -std=c11 -ffp-contract=off -fPIC -shared (oracle/Makefile).
 * -ffp-contract=off matches the reference's -std=c++11 ISO mode
 * (CMakeLists.txt:10-19; GCC disables FMA contraction in ISO modes).
 */
#include "orbx_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static const int kPattern[256 * 4] = {
#include "../orbslam2commentedbyxcm_amd/csrc/orb_pattern.inc"
};

/* ORBextractor.cc:44-46 */
enum { PATCH_SIZE = 31, HALF_PATCH_SIZE = 15, EDGE_THRESHOLD = 19 };

/* ---------------------------------------------------------------- cv helpers */

/* cvRound: SSE2 cvtsd2si / cvtss2si under the default round-to-nearest-even mode. */
int ora_cv_round(double v) { return (int)lrint(v); }
int ora_cv_roundf(float v) { return (int)lrintf(v); }
static int cv_floorf(float v) { return (int)floorf(v); }

/* cv::fastAtan2 (OpenCV 3.3.1 core/mathfuncs_core: atanImpl<float>), degrees [0,360).
 * Called at ORBextractor.cc:105. */
float ora_fast_atan2(float y, float x) {
    const float deg = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * deg;
    const float p3 = -0.3258083974640975f * deg;
    const float p5 = 0.1555786518463281f * deg;
    const float p7 = -0.04432655554792128f * deg;
    const float eps = (float)2.2204460492503131e-16; /* (float)DBL_EPSILON */
    float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

/* ---------------------------------------------------------------- parameters */

/* ORBextractor::ORBextractor, ORBextractor.cc:438-550 */
int ora_params_init(ora_params* p, int nfeatures, float scale_factor, int nlevels,
                    int ini_th_fast, int min_th_fast) {
    if (!p || nlevels < 1 || nlevels > ORA_MAX_LEVELS) return -1;
    memset(p, 0, sizeof(*p));
    p->nfeatures = nfeatures;
    p->scale_factor = (double)scale_factor; /* member is double (ORBextractor.h:207) */
    p->nlevels = nlevels;
    p->ini_th_fast = ini_th_fast;
    p->min_th_fast = min_th_fast;

    /* cc:452-461: float accumulator times double member */
    p->scale[0] = 1.0f;
    p->sigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
        p->scale[i] = (float)((double)p->scale[i - 1] * p->scale_factor);
        p->sigma2[i] = p->scale[i] * p->scale[i];
    }
    /* cc:466-470 */
    for (int i = 0; i < nlevels; i++) {
        p->inv_scale[i] = 1.0f / p->scale[i];
        p->inv_sigma2[i] = 1.0f / p->sigma2[i];
    }
    /* cc:480-500 */
    float factor = (float)(1.0f / p->scale_factor);
    float nDesired = (float)nfeatures * (1 - factor) /
                     (1 - (float)pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int level = 0; level < nlevels - 1; level++) {
        p->features_per_level[level] = ora_cv_roundf(nDesired);
        sum += p->features_per_level[level];
        nDesired *= factor;
    }
    p->features_per_level[nlevels - 1] = nfeatures - sum > 0 ? nfeatures - sum : 0;

    /* cc:519-549: circular patch row half-widths */
    int vmax = cv_floorf(HALF_PATCH_SIZE * sqrtf(2.f) / 2 + 1);
    int vmin = (int)ceilf(HALF_PATCH_SIZE * sqrtf(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    int v, v0;
    for (v = 0; v <= vmax; ++v) p->umax[v] = ora_cv_round(sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (p->umax[v0] == p->umax[v0 + 1]) ++v0;
        p->umax[v] = v0;
        ++v0;
    }
    return 0;
}

/* ComputePyramid level size, ORBextractor.cc:1641-1643 */
void ora_level_size(const ora_params* p, int W, int H, int level, int* w, int* h) {
    float s = p->inv_scale[level];
    *w = ora_cv_roundf((float)W * s);
    *h = ora_cv_roundf((float)H * s);
}

/* ---------------------------------------------------------------- resize */

/* cv::resize(src, dst, dsize, 0, 0, INTER_LINEAR) for CV_8UC1, OpenCV 3.3.1
 * imgproc/resize.cpp (non-IPP): float source coordinates, 11-bit fixed-point
 * coefficients (INTER_RESIZE_COEF_SCALE = 2048), exact integer horizontal pass,
 * and the VResizeLinear<uchar,...> vertical pass
 *   dst = ((b0*(S0>>4))>>16 + (b1*(S1>>4))>>16 + 2) >> 2
 * (identical in its SSE2 and scalar forms).  Called at ORBextractor.cc:1656-1661. */
void ora_resize_linear_u8(const uint8_t* src, int sw, int sh, size_t sstride,
                          uint8_t* dst, int dw, int dh, size_t dstride) {
    double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    int* xofs = (int*)malloc(sizeof(int) * (size_t)dw);
    short* ialpha = (short*)malloc(sizeof(short) * 2 * (size_t)dw);
    int* hrow0 = (int*)malloc(sizeof(int) * (size_t)dw);
    int* hrow1 = (int*)malloc(sizeof(int) * (size_t)dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floorf(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        float c0 = 1.f - fx, c1 = fx;
        ialpha[2 * dx] = (short)ora_cv_roundf(c0 * 2048);
        ialpha[2 * dx + 1] = (short)ora_cv_roundf(c1 * 2048);
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floorf(fy);
        fy -= sy;
        short b0 = (short)ora_cv_roundf((1.f - fy) * 2048);
        short b1 = (short)ora_cv_roundf(fy * 2048);
        /* resizeGeneric_Invoker: rows sy, sy+1 clipped to [0, sh-1] */
        int r0 = sy < 0 ? 0 : (sy >= sh ? sh - 1 : sy);
        int r1 = sy + 1 < 0 ? 0 : (sy + 1 >= sh ? sh - 1 : sy + 1);
        const uint8_t* S0 = src + (size_t)r0 * sstride;
        const uint8_t* S1 = src + (size_t)r1 * sstride;
        for (int dx = 0; dx < dw; dx++) {
            int sx = xofs[dx];
            if (dx < xmax) {
                int a0 = ialpha[2 * dx], a1 = ialpha[2 * dx + 1];
                hrow0[dx] = S0[sx] * a0 + S0[sx + 1] * a1;
                hrow1[dx] = S1[sx] * a0 + S1[sx + 1] * a1;
            } else {
                hrow0[dx] = S0[sx] * 2048;
                hrow1[dx] = S1[sx] * 2048;
            }
        }
        uint8_t* D = dst + (size_t)dy * dstride;
        for (int dx = 0; dx < dw; dx++) {
            int v = (((b0 * (hrow0[dx] >> 4)) >> 16) + ((b1 * (hrow1[dx] >> 4)) >> 16) + 2) >> 2;
            D[dx] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    }
    free(xofs);
    free(ialpha);
    free(hrow0);
    free(hrow1);
}

/* ---------------------------------------------------------------- Gaussian blur */

static int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

/* cv::GaussianBlur(m, m, Size(7,7), 2, 2, BORDER_REFLECT_101) on CV_8UC1, OpenCV 3.3.1
 * non-IPP fixed-point path: the float kernel exp(-x^2/8)/sum is scaled by 256 and
 * rounded to {18,34,49,55,49,34,18} (sum 257), integer row pass, integer column
 * pass with (sum + 2^15) >> 16 and saturation.  Called at ORBextractor.cc:1587-1595
 * on a clone of the level ROI, so the border reflects around the ROI itself. */
void ora_gaussian_blur7_u8(const uint8_t* src, int w, int h, size_t sstride,
                           uint8_t* dst, size_t dstride) {
    static const int K[7] = {18, 34, 49, 55, 49, 34, 18};
    int* rows = (int*)malloc(sizeof(int) * (size_t)w * (size_t)h);
    for (int y = 0; y < h; y++) {
        const uint8_t* s = src + (size_t)y * sstride;
        for (int x = 0; x < w; x++) {
            int acc = 0;
            for (int k = -3; k <= 3; k++) acc += K[k + 3] * s[reflect101(x + k, w)];
            rows[(size_t)y * w + x] = acc;
        }
    }
    for (int y = 0; y < h; y++) {
        uint8_t* d = dst + (size_t)y * dstride;
        for (int x = 0; x < w; x++) {
            int acc = 0;
            for (int k = -3; k <= 3; k++) acc += K[k + 3] * rows[(size_t)reflect101(y + k, h) * w + x];
            int v = (acc + (1 << 15)) >> 16;
            d[x] = (uint8_t)(v > 255 ? 255 : v);
        }
    }
    free(rows);
}

/* ---------------------------------------------------------------- FAST-9/16 */

/* features2d/fast_score.cpp makeOffsets(pixel, step, 16): ring as (dx, dy) */
static const int kRing[16][2] = {{0, 3},  {1, 3},   {2, 2},   {3, 1},   {3, 0},  {3, -1},
                                 {2, -2}, {1, -3},  {0, -3},  {-1, -3}, {-2, -2}, {-3, -1},
                                 {-3, 0}, {-3, 1},  {-2, 2},  {-1, 3}};

static void make_offsets(int pixel[25], int stride) {
    for (int k = 0; k < 16; k++) pixel[k] = kRing[k][0] + kRing[k][1] * stride;
    for (int k = 16; k < 25; k++) pixel[k] = pixel[k - 16];
}

/* cornerScore<16> (features2d/fast_score.cpp, scalar form) */
static int corner_score16(const uint8_t* ptr, const int pixel[25], int threshold) {
    const int K = 8, N = K * 3 + 1;
    int k, v = ptr[0];
    short d[25];
    for (k = 0; k < N; k++) d[k] = (short)(v - ptr[pixel[k]]);
    int a0 = threshold;
    for (k = 0; k < 16; k += 2) {
        int a = d[k + 1] < d[k + 2] ? d[k + 1] : d[k + 2];
        if (d[k + 3] < a) a = d[k + 3];
        if (a <= a0) continue;
        for (int q = 4; q <= 8; q++)
            if (d[k + q] < a) a = d[k + q];
        int t = a < d[k] ? a : d[k];
        if (t > a0) a0 = t;
        t = a < d[k + 9] ? a : d[k + 9];
        if (t > a0) a0 = t;
    }
    int b0 = -a0;
    for (k = 0; k < 16; k += 2) {
        int b = d[k + 1] > d[k + 2] ? d[k + 1] : d[k + 2];
        for (int q = 3; q <= 5; q++)
            if (d[k + q] > b) b = d[k + q];
        if (b >= b0) continue;
        for (int q = 6; q <= 8; q++)
            if (d[k + q] > b) b = d[k + q];
        int t = b > d[k] ? b : d[k];
        if (t < b0) b0 = t;
        t = b > d[k + 9] ? b : d[k + 9];
        if (t < b0) b0 = t;
    }
    return -b0 - 1;
}

int ora_fast_corner_score(const uint8_t* p, int stride, int threshold) {
    int pixel[25];
    make_offsets(pixel, stride);
    return corner_score16(p, pixel, threshold);
}

/* cv::FAST(img, kps, threshold, true) == FAST_t<16> with non-max suppression
 * (features2d/fast.cpp, scalar form; its SSE2 block detects the same set).
 * Called per cell at ORBextractor.cc:1091-1104.  Returns the keypoint count, or -1
 * on overflow.  Keypoints: (x=j, y=i, size 7, angle -1, response=score) in raster order. */
int ora_fast_detect(const uint8_t* img, int rows, int cols, size_t stride, int threshold,
                    ora_keypoint* out, int cap) {
    const int K = 8, N = 25;
    int pixel[25];
    int i, j, k, nout = 0;
    make_offsets(pixel, (int)stride);
    if (threshold < 0) threshold = 0;
    if (threshold > 255) threshold = 255;
    if (rows < 7 || cols < 7) return 0;
    uint8_t tab[512];
    for (i = -255; i <= 255; i++) tab[i + 255] = (uint8_t)(i < -threshold ? 1 : i > threshold ? 2 : 0);

    uint8_t* buf = (uint8_t*)calloc((size_t)cols * 3, 1);
    int* cp = (int*)malloc(sizeof(int) * (size_t)(cols + 1) * 3);
    uint8_t* bufs[3] = {buf, buf + cols, buf + 2 * cols};
    int* cpbuf[3] = {cp + 1, cp + 1 + (cols + 1), cp + 1 + 2 * (cols + 1)};

    for (i = 3; i < rows - 2; i++) {
        const uint8_t* ptr = img + (size_t)i * stride + 3;
        uint8_t* curr = bufs[(i - 3) % 3];
        int* cornerpos = cpbuf[(i - 3) % 3];
        memset(curr, 0, (size_t)cols);
        int ncorners = 0;
        if (i < rows - 3) {
            for (j = 3; j < cols - 3; j++, ptr++) {
                int v = ptr[0];
                const uint8_t* t = tab - v + 255;
                int d = t[ptr[pixel[0]]] | t[ptr[pixel[8]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[2]]] | t[ptr[pixel[10]]];
                d &= t[ptr[pixel[4]]] | t[ptr[pixel[12]]];
                d &= t[ptr[pixel[6]]] | t[ptr[pixel[14]]];
                if (d == 0) continue;
                d &= t[ptr[pixel[1]]] | t[ptr[pixel[9]]];
                d &= t[ptr[pixel[3]]] | t[ptr[pixel[11]]];
                d &= t[ptr[pixel[5]]] | t[ptr[pixel[13]]];
                d &= t[ptr[pixel[7]]] | t[ptr[pixel[15]]];
                if (d & 1) {
                    int vt = v - threshold, count = 0;
                    for (k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x < vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
                if (d & 2) {
                    int vt = v + threshold, count = 0;
                    for (k = 0; k < N; k++) {
                        int x = ptr[pixel[k]];
                        if (x > vt) {
                            if (++count > K) {
                                cornerpos[ncorners++] = j;
                                curr[j] = (uint8_t)corner_score16(ptr, pixel, threshold);
                                break;
                            }
                        } else
                            count = 0;
                    }
                }
            }
        }
        cornerpos[-1] = ncorners;
        if (i == 3) continue;
        const uint8_t* prev = bufs[(i - 4 + 3) % 3];
        const uint8_t* pprev = bufs[(i - 5 + 3) % 3];
        cornerpos = cpbuf[(i - 4 + 3) % 3];
        ncorners = cornerpos[-1];
        for (k = 0; k < ncorners; k++) {
            j = cornerpos[k];
            int score = prev[j];
            if (score > prev[j + 1] && score > prev[j - 1] && score > pprev[j - 1] &&
                score > pprev[j] && score > pprev[j + 1] && score > curr[j - 1] &&
                score > curr[j] && score > curr[j + 1]) {
                if (nout >= cap) { nout = -1; goto done; }
                ora_keypoint* kp = &out[nout++];
                kp->x = (float)j;
                kp->y = (float)(i - 1);
                kp->size = 7.f;
                kp->angle = -1.f;
                kp->response = (float)score;
                kp->octave = 0;
                kp->class_id = -1;
            }
        }
    }
done:
    free(buf);
    free(cp);
    return nout;
}

/* ---------------------------------------------------------------- orientation / rBRIEF */

/* IC_Angle, ORBextractor.cc:59-106 */
float ora_ic_angle(const uint8_t* img, size_t stride, float x, float y, const int* umax) {
    int m_01 = 0, m_10 = 0;
    const uint8_t* center = img + (size_t)ora_cv_roundf(y) * stride + ora_cv_roundf(x);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * center[u];
    int step = (int)stride;
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0;
        int d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int val_plus = center[u + v * step], val_minus = center[u - v * step];
            v_sum += (val_plus - val_minus);
            m_10 += u * (val_plus + val_minus);
        }
        m_01 += v * v_sum;
    }
    return ora_fast_atan2((float)m_01, (float)m_10);
}

/* ORBextractor.cc:109, 123-125: angle (deg, float) -> radians (float) -> cos/sin.
 * The reference calls std::cos(float) (glibc cosf); this restatement fixes the
 * result to the correctly rounded float value, (float)cos((double)r).  glibc 2.35's
 * cosf/sinf differ from it by one ulp on 0.26 % / 0.55 % of [0,360) degrees
 * (measured).
 *
 * ora_set_trig_mode(1) switches the calling thread to the reference's literal
 * arithmetic, cosf / sinf of the float radian (ORBextractor.cc:123-125 under `using
 * namespace std`), so the descriptor-level effect of H3 can be counted
 * (tests/h3_flip_count.py).  Mode 0 (default) is the shipped restatement. */
static _Thread_local int g_trig_mode = 0;

void ora_set_trig_mode(int mode) { g_trig_mode = mode; }

void ora_cos_sin(float angle_deg, float* c, float* s) {
    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    float r = angle_deg * factorPI;
    if (g_trig_mode == 1) {
        *c = cosf(r);
        *s = sinf(r);
        return;
    }
    *c = (float)cos((double)r);
    *s = (float)sin((double)r);
}

/* Hazard H4 at descriptor level.  The reference is built by g++ -O3 -march=native
 * (CMakeLists.txt:10-19), and g++ contracts a*b + c*d into fma(a, b, c*d) in C++ even
 * under -std=c++11 (GCC keeps contraction off by default only for ISO C): the
 * reference's own BowVector.cpp built with DBoW2's flags holds a vfmadd
 * (tests/test_vocab_ref.py).  The sample offsets x*b + y*a and x*a - y*b
 * (ORBextractor.cc:136-138) are such expressions, and GCC's FMA pass fuses the first
 * product into the add: fma(x, b, y*a), fma(x, a, -(y*b)).  That is the shipped form
 * (here and in k_describe).  ora_set_contract_mode(0) switches the calling thread to the
 * unfused form, so the effect can be counted (tests/h4_contract_count.py: 3 of 257,543
 * descriptors at configs[1]). */
static _Thread_local int g_contract_mode = 1;

void ora_set_contract_mode(int mode) { g_contract_mode = mode; }

static inline float brief_u(float x, float y, float a, float b) {
    return g_contract_mode ? fmaf(x, b, y * a) : x * b + y * a;
}
static inline float brief_v(float x, float y, float a, float b) {
    return g_contract_mode ? fmaf(x, a, -(y * b)) : x * a - y * b;
}

/* computeOrbDescriptor, ORBextractor.cc:118-172 (pattern: cc:176-434) */
void ora_orb_descriptor(const uint8_t* img, size_t stride, float x, float y, float angle_deg,
                        uint8_t* desc) {
    float a, b;
    ora_cos_sin(angle_deg, &a, &b);
    const uint8_t* center = img + (size_t)ora_cv_roundf(y) * stride + ora_cv_roundf(x);
    const int step = (int)stride;
    const int* pattern = kPattern;
    for (int i = 0; i < 32; ++i, pattern += 32) {
        int val = 0;
        for (int j = 0; j < 8; j++) {
            const int* p0 = pattern + 4 * j;       /* point 2j   : (x, y) */
            const int* p1 = pattern + 4 * j + 2;   /* point 2j+1 */
            float x0 = (float)p0[0], y0 = (float)p0[1], x1 = (float)p1[0], y1 = (float)p1[1];
            int t0 = center[ora_cv_roundf(brief_u(x0, y0, a, b)) * step + ora_cv_roundf(brief_v(x0, y0, a, b))];
            int t1 = center[ora_cv_roundf(brief_u(x1, y1, a, b)) * step + ora_cv_roundf(brief_v(x1, y1, a, b))];
            val |= (t0 < t1) << j;
        }
        desc[i] = (uint8_t)val;
    }
}

/* ---------------------------------------------------------------- octree */

typedef struct ora_node {
    int ulx, uly, urx, ury, blx, bly, brx, bry; /* UL, UR, BL, BR corners (ORBextractor.h:60) */
    int* keys;                                  /* indices into the level's candidate array */
    int nkeys;
    int no_more;                                /* bNoMore (ORBextractor.h:67) */
    long seq;                                   /* allocation order (hazard H1) */
    struct ora_node *prev, *next;
} ora_node;

typedef struct {
    ora_node *head, *tail;
    int size;
    long next_seq;
} ora_list;

static ora_node* list_insert_copy(ora_list* L, const ora_node* src, int front) {
    ora_node* n = (ora_node*)malloc(sizeof(ora_node));
    *n = *src;
    n->seq = L->next_seq++;
    if (front) {
        n->prev = NULL;
        n->next = L->head;
        if (L->head) L->head->prev = n; else L->tail = n;
        L->head = n;
    } else {
        n->next = NULL;
        n->prev = L->tail;
        if (L->tail) L->tail->next = n; else L->head = n;
        L->tail = n;
    }
    L->size++;
    return n;
}

static ora_node* list_erase(ora_list* L, ora_node* n) {
    ora_node* nx = n->next;
    if (n->prev) n->prev->next = n->next; else L->head = n->next;
    if (n->next) n->next->prev = n->prev; else L->tail = n->prev;
    L->size--;
    free(n->keys);
    free(n);
    return nx;
}

/* ExtractorNode::DivideNode, ORBextractor.cc:581-653 */
static void divide_node(const ora_node* p, const ora_keypoint* keys, ora_node c[4]) {
    const int halfX = (int)ceilf((float)(p->urx - p->ulx) / 2);
    const int halfY = (int)ceilf((float)(p->bry - p->uly) / 2);
    memset(c, 0, 4 * sizeof(ora_node));
    c[0].ulx = p->ulx;         c[0].uly = p->uly;
    c[0].urx = p->ulx + halfX; c[0].ury = p->uly;
    c[0].blx = p->ulx;         c[0].bly = p->uly + halfY;
    c[0].brx = p->ulx + halfX; c[0].bry = p->uly + halfY;

    c[1].ulx = c[0].urx;       c[1].uly = c[0].ury;
    c[1].urx = p->urx;         c[1].ury = p->ury;
    c[1].blx = c[0].brx;       c[1].bly = c[0].bry;
    c[1].brx = p->urx;         c[1].bry = p->uly + halfY;

    c[2].ulx = c[0].blx;       c[2].uly = c[0].bly;
    c[2].urx = c[0].brx;       c[2].ury = c[0].bry;
    c[2].blx = p->blx;         c[2].bly = p->bly;
    c[2].brx = c[0].brx;       c[2].bry = p->bly;

    c[3].ulx = c[2].urx;       c[3].uly = c[2].ury;
    c[3].urx = c[1].brx;       c[3].ury = c[1].bry;
    c[3].blx = c[2].brx;       c[3].bly = c[2].bry;
    c[3].brx = p->brx;         c[3].bry = p->bry;

    for (int q = 0; q < 4; q++) c[q].keys = (int*)malloc(sizeof(int) * (size_t)(p->nkeys ? p->nkeys : 1));
    for (int i = 0; i < p->nkeys; i++) {
        const ora_keypoint* kp = &keys[p->keys[i]];
        int q;
        if (kp->x < (float)c[0].urx)
            q = kp->y < (float)c[0].bry ? 0 : 2;
        else
            q = kp->y < (float)c[0].bry ? 1 : 3;
        c[q].keys[c[q].nkeys++] = p->keys[i];
    }
    for (int q = 0; q < 4; q++)
        if (c[q].nkeys == 1) c[q].no_more = 1;
}

typedef struct { int size; ora_node* node; } size_ptr;

/* Hazard H1.  std::sort on pair<int, ExtractorNode*> (ORBextractor.cc:899-913) orders equal
 * sizes by node address, i.e. by the heap.  Mode 0 (shipped, = the GPU): allocation order,
 * what a monotonic allocator gives -- the later-created node sorts last and is split first.
 * Mode 1 (measurement only, tests/h1_tie_count.py): the opposite, earlier-created first.
 * g_octree_ties counts, per thread, final-phase passes in which a split node shared its
 * size with another node of the pass (the order then depends on the tie-break). */
static _Thread_local int g_octree_tie_mode = 0;
static _Thread_local long g_octree_ties = 0;

void ora_set_octree_tie_mode(int mode) { g_octree_tie_mode = mode; }
long ora_octree_ties(int reset) {
    const long t = g_octree_ties;
    if (reset) g_octree_ties = 0;
    return t;
}

static int cmp_size_ptr(const void* a, const void* b) {
    const size_ptr* x = (const size_ptr*)a;
    const size_ptr* y = (const size_ptr*)b;
    if (x->size != y->size) return x->size < y->size ? -1 : 1;
    const int later = x->node->seq < y->node->seq ? -1 : (x->node->seq > y->node->seq ? 1 : 0);
    return g_octree_tie_mode ? -later : later;
}

/* Push the non-empty children n1..n4 to the list front; record those with >1 key. */
static void push_children(ora_list* L, ora_node c[4], size_ptr* vsz, int* nvsz) {
    for (int q = 0; q < 4; q++) {
        if (c[q].nkeys > 0) {
            ora_node* n = list_insert_copy(L, &c[q], 1);
            if (c[q].nkeys > 1) {
                vsz[*nvsz].size = c[q].nkeys;
                vsz[*nvsz].node = n;
                (*nvsz)++;
            }
        } else {
            free(c[q].keys);
        }
    }
}

/* ORBextractor::DistributeOctTree, ORBextractor.cc:667-1013.  Returns the number of
 * keypoints written (list order), or -1 if cap is too small. */
int ora_distribute_octree(const ora_keypoint* keys, int n, int minX, int maxX, int minY,
                          int maxY, int N, ora_keypoint* out, int cap) {
    const int nIni = (int)roundf((float)(maxX - minX) / (float)(maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    ora_list L = {NULL, NULL, 0, 0};
    ora_node** ini = (ora_node**)malloc(sizeof(ora_node*) * (size_t)nIni);
    for (int i = 0; i < nIni; i++) {
        ora_node ni;
        memset(&ni, 0, sizeof(ni));
        ni.ulx = (int)(hX * (float)i);       ni.uly = 0;
        ni.urx = (int)(hX * (float)(i + 1)); ni.ury = 0;
        ni.blx = ni.ulx;                     ni.bly = maxY - minY;
        ni.brx = ni.urx;                     ni.bry = maxY - minY;
        ni.keys = (int*)malloc(sizeof(int) * (size_t)(n ? n : 1));
        ini[i] = list_insert_copy(&L, &ni, 0);
    }
    for (int i = 0; i < n; i++) {
        size_t idx = (size_t)(keys[i].x / hX);
        ini[idx]->keys[ini[idx]->nkeys++] = i;
    }
    free(ini);
    for (ora_node* it = L.head; it;) {
        if (it->nkeys == 1) {
            it->no_more = 1;
            it = it->next;
        } else if (it->nkeys == 0)
            it = list_erase(&L, it);
        else
            it = it->next;
    }

    /* At most 4 children per divided node; a pass divides at most L.size nodes. */
    size_t vcap = 4 * (size_t)(n + 8);
    size_ptr* vsz = (size_ptr*)malloc(sizeof(size_ptr) * vcap);
    size_ptr* vprev = (size_ptr*)malloc(sizeof(size_ptr) * vcap);
    int nvsz = 0;
    int finish = 0;
    while (!finish) {
        int prevSize = L.size;
        int nToExpand = 0;
        nvsz = 0;
        for (ora_node* it = L.head; it;) {
            if (it->no_more) { it = it->next; continue; }
            ora_node c[4];
            divide_node(it, keys, c);
            int before = nvsz;
            push_children(&L, c, vsz, &nvsz);
            nToExpand += nvsz - before;
            it = list_erase(&L, it);
        }
        if (L.size >= N || L.size == prevSize) {
            finish = 1;
        } else if (L.size + nToExpand * 3 > N) {
            while (!finish) {
                prevSize = L.size;
                int nprev = nvsz;
                memcpy(vprev, vsz, sizeof(size_ptr) * (size_t)nprev);
                nvsz = 0;
                qsort(vprev, (size_t)nprev, sizeof(size_ptr), cmp_size_ptr);
                int jstop = 0;
                for (int j = nprev - 1; j >= 0; j--) {
                    ora_node c[4];
                    divide_node(vprev[j].node, keys, c);
                    push_children(&L, c, vsz, &nvsz);
                    list_erase(&L, vprev[j].node);
                    jstop = j;
                    if (L.size >= N) break;
                }
                /* a tie decides the order if a split node (index >= jstop) has a neighbour
                 * of equal size in the sorted pass */
                for (int j = jstop; j < nprev; j++)
                    if ((j > 0 && vprev[j - 1].size == vprev[j].size) ||
                        (j + 1 < nprev && vprev[j + 1].size == vprev[j].size)) {
                        g_octree_ties++;
                        break;
                    }
                if (L.size >= N || L.size == prevSize) finish = 1;
            }
        }
    }
    free(vsz);
    free(vprev);

    /* cc:984-1009: keep the max-response key of each node (first wins ties) */
    int nout = 0;
    for (ora_node* it = L.head; it; it = it->next) {
        if (nout >= cap) { nout = -1; break; }
        int best = it->keys[0];
        float maxResponse = keys[best].response;
        for (int k = 1; k < it->nkeys; k++) {
            if (keys[it->keys[k]].response > maxResponse) {
                best = it->keys[k];
                maxResponse = keys[best].response;
            }
        }
        out[nout++] = keys[best];
    }
    while (L.head) list_erase(&L, L.head);
    return nout;
}

/* ---------------------------------------------------------------- pipeline */

/* ComputePyramid, ORBextractor.cc:1635-1694 (interiors only; the REFLECT_101 border
 * is never read by extraction -- App. B3 of SURVEY.md). */
int ora_pyramid(const ora_params* p, const uint8_t* img, int W, int H, size_t stride,
                uint8_t** levels) {
    int pw = W, ph = H;
    for (int level = 0; level < p->nlevels; ++level) {
        int w, h;
        ora_level_size(p, W, H, level, &w, &h);
        if (level == 0) {
            for (int y = 0; y < h; y++) memcpy(levels[0] + (size_t)y * w, img + (size_t)y * stride, (size_t)w);
        } else {
            ora_resize_linear_u8(levels[level - 1], pw, ph, (size_t)pw, levels[level], w, h, (size_t)w);
        }
        pw = w;
        ph = h;
    }
    return 0;
}

/* ComputeKeyPointsOctTree cell loop, ORBextractor.cc:1025-1122 */
static int level_candidates(const ora_params* p, const uint8_t* level, int w, int h, ora_keypoint* out,
                            int cap, int* cell_counts, int cell_cap, int* ncells);

int ora_level_candidates(const ora_params* p, const uint8_t* level, int w, int h, ora_keypoint* out,
                         int cap) {
    return level_candidates(p, level, w, h, out, cap, NULL, 0, NULL);
}

/* The same, plus the FAST output count of every visited cell in visit order (test
 * infrastructure for the H1 allocator measurement, tests/h1_glibc_measure.py). */
int ora_level_candidates_cells(const ora_params* p, const uint8_t* level, int w, int h, ora_keypoint* out,
                               int cap, int* cell_counts, int cell_cap, int* ncells) {
    return level_candidates(p, level, w, h, out, cap, cell_counts, cell_cap, ncells);
}

static int level_candidates(const ora_params* p, const uint8_t* level, int w, int h, ora_keypoint* out,
                            int cap, int* cell_counts, int cell_cap, int* ncells) {
    const float Wc = 30;
    const int minBorderX = EDGE_THRESHOLD - 3;
    const int minBorderY = minBorderX;
    const int maxBorderX = w - EDGE_THRESHOLD + 3;
    const int maxBorderY = h - EDGE_THRESHOLD + 3;
    const float width = (float)(maxBorderX - minBorderX);
    const float height = (float)(maxBorderY - minBorderY);
    const int nCols = (int)(width / Wc);
    const int nRows = (int)(height / Wc);
    const int wCell = (int)ceilf(width / nCols);
    const int hCell = (int)ceilf(height / nRows);
    ora_keypoint cell[64 * 64];
    int nout = 0;
    for (int i = 0; i < nRows; i++) {
        const float iniY = (float)(minBorderY + i * hCell);
        float maxY = iniY + hCell + 6;
        if (iniY >= maxBorderY - 3) continue;
        if (maxY > maxBorderY) maxY = (float)maxBorderY;
        for (int j = 0; j < nCols; j++) {
            const float iniX = (float)(minBorderX + j * wCell);
            float maxX = iniX + wCell + 6;
            if (iniX >= maxBorderX - 6) continue;
            if (maxX > maxBorderX) maxX = (float)maxBorderX;
            const int y0 = (int)iniY, x0 = (int)iniX;
            const int rows = (int)maxY - y0, cols = (int)maxX - x0;
            const uint8_t* sub = level + (size_t)y0 * w + x0;
            int nc = ora_fast_detect(sub, rows, cols, (size_t)w, p->ini_th_fast, cell, 64 * 64);
            if (nc == 0) nc = ora_fast_detect(sub, rows, cols, (size_t)w, p->min_th_fast, cell, 64 * 64);
            if (nc < 0) return -1;
            if (ncells) {
                if (*ncells >= cell_cap) return -1;
                cell_counts[(*ncells)++] = nc;
            }
            for (int k = 0; k < nc; k++) {
                if (nout >= cap) return -1;
                out[nout] = cell[k];
                out[nout].x += (float)(j * wCell);
                out[nout].y += (float)(i * hCell);
                nout++;
            }
        }
    }
    return nout;
}

/* ORBextractor::operator(), ORBextractor.cc:1513-1629 */
int ora_extract(const ora_params* p, const uint8_t* img, int W, int H, size_t stride,
                ora_keypoint* kps, uint8_t* desc, int cap, int* level_counts) {
    if (W <= 0 || H <= 0) return 0;
    const int L = p->nlevels;
    int lw[ORA_MAX_LEVELS], lh[ORA_MAX_LEVELS];
    uint8_t* levels[ORA_MAX_LEVELS];
    for (int l = 0; l < L; l++) {
        ora_level_size(p, W, H, l, &lw[l], &lh[l]);
        levels[l] = (uint8_t*)malloc((size_t)lw[l] * lh[l]);
    }
    ora_pyramid(p, img, W, H, stride, levels);

    ora_keypoint* all[ORA_MAX_LEVELS];
    int nlev[ORA_MAX_LEVELS];
    int total = 0, rc = 0;
    const int candcap = 1 << 20;
    ora_keypoint* cand = (ora_keypoint*)malloc(sizeof(ora_keypoint) * (size_t)candcap);
    for (int l = 0; l < L; l++) {
        all[l] = NULL;
        nlev[l] = 0;
    }
    for (int l = 0; l < L && rc == 0; l++) {
        const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
        const int maxBorderX = lw[l] - EDGE_THRESHOLD + 3, maxBorderY = lh[l] - EDGE_THRESHOLD + 3;
        int nc = ora_level_candidates(p, levels[l], lw[l], lh[l], cand, candcap);
        if (nc < 0) { rc = -1; break; }
        int kcap = nc + 8;
        all[l] = (ora_keypoint*)malloc(sizeof(ora_keypoint) * (size_t)kcap);
        int nk = ora_distribute_octree(cand, nc, minBorderX, maxBorderX, minBorderY, maxBorderY,
                                       p->features_per_level[l], all[l], kcap);
        if (nk < 0) { rc = -1; break; }
        /* cc:1140-1155 */
        const int scaledPatchSize = (int)(PATCH_SIZE * p->scale[l]);
        for (int i = 0; i < nk; i++) {
            all[l][i].x += minBorderX;
            all[l][i].y += minBorderY;
            all[l][i].octave = l;
            all[l][i].size = (float)scaledPatchSize;
        }
        /* cc:1160-1163 */
        for (int i = 0; i < nk; i++)
            all[l][i].angle = ora_ic_angle(levels[l], (size_t)lw[l], all[l][i].x, all[l][i].y, p->umax);
        nlev[l] = nk;
        total += nk;
    }
    free(cand);
    if (rc == 0 && total > cap) rc = -1;
    if (rc == 0) {
        int offset = 0;
        for (int l = 0; l < L; l++) {
            int nk = nlev[l];
            if (level_counts) level_counts[l] = nk;
            if (nk == 0) continue;
            uint8_t* blurred = (uint8_t*)malloc((size_t)lw[l] * lh[l]);
            ora_gaussian_blur7_u8(levels[l], lw[l], lh[l], (size_t)lw[l], blurred, (size_t)lw[l]);
            for (int i = 0; i < nk; i++)
                ora_orb_descriptor(blurred, (size_t)lw[l], all[l][i].x, all[l][i].y, all[l][i].angle,
                                   desc + (size_t)(offset + i) * 32);
            free(blurred);
            if (l != 0) {
                float scale = p->scale[l];
                for (int i = 0; i < nk; i++) {
                    all[l][i].x = all[l][i].x * scale;
                    all[l][i].y = all[l][i].y * scale;
                }
            }
            memcpy(kps + offset, all[l], sizeof(ora_keypoint) * (size_t)nk);
            offset += nk;
        }
        rc = total;
    }
    for (int l = 0; l < L; l++) {
        free(levels[l]);
        free(all[l]);
    }
    return rc;
}

/* ORBmatcher::DescriptorDistance, ORBmatcher.cc:1983-2003 (SWAR popcount over 8 x int32) */
int ora_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t va, vb;
        memcpy(&va, a + 4 * i, 4);
        memcpy(&vb, b + 4 * i, 4);
        uint32_t v = va ^ vb;
        v = v - ((v >> 1) & 0x55555555u);
        v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0Fu) * 0x1010101u) >> 24);
    }
    return dist;
}
