// orbx_extract.hip -- MI355X (gfx950) kernels for ORB-SLAM2's ORBextractor::operator().
//
// Pipeline for a batch of B frames of one size (one launch per stage; every stage
// covers all frames and all levels at once):
//   1. k_pyramid     : image pyramid, one tile of every level per workgroup   cc:1635-1694
//   2. k_level_tiles : GaussianBlur 7x7 sigma 2 REFLECT_101 + FAST strength map
//                                                                 cc:1587-1595, 1091-1104
//   3. k_fast_cells  : per 30-px cell FAST-9 threshold, window-local NMS, iniTh -> minTh
//                      fallback, ordered compaction                   cc:1025-1122
//   4. k_octree      : DistributeOctTree, one workgroup per (frame, level)  cc:667-1013
//   5. k_describe    : IC angle + steered BRIEF + level scaling + output   cc:59-172, 1597-1627
// Bit-exactness: integer arithmetic everywhere except fastAtan2/cos/sin/cvRound,
// which follow the reference's float expression order (built -ffp-contract=off).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <type_traits>

#include "orbx_error.h"
#include "orbx_kernels.h"
#include "orbx_sincos.h"

namespace orbx {

const char* const kStageNames[kStages] = {"pyramid", "score_blur", "fast_cells", "octree", "describe", "total"};

// the 256 rBRIEF point pairs (x0, y0, x1, y1 as int8, one int per pair), ordered
// lane-major for k_describe: c_pattern[ql][k] = pair ql + 16 k, so quarter lane ql's
// 16 pairs are four 16-byte loads
__constant__ __align__(16) int c_pattern[16][16];

__constant__ int c_umax[16];
// IC_Angle by rows: for a patch row v and the patch's start alignment d0 = (x-15) & 3,
// c_icm[d0][|v|] holds 9 dwords of byte masks (1 where |u| <= umax[|v|]) and c_icw the
// same bytes weighted by u + 15, laid over the 36 bytes staged from (x-15) & ~3.
__constant__ __align__(16) uint32_t c_icm[4][16][12];
__constant__ __align__(16) uint32_t c_icw[4][16][12];

static const int8_t kPatternHost[1024] = {
#include "orb_pattern.inc"
};

hipError_t upload_constants(const OrbParams& prm) {
    int patq[16][16];
    for (int ql = 0; ql < 16; ql++)
        for (int k = 0; k < 16; k++) memcpy(&patq[ql][k], kPatternHost + 4 * (ql + 16 * k), 4);
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_pattern), patq, sizeof(patq));
    if (e != hipSuccess) return e;
    uint32_t icm[4][16][12] = {}, icw[4][16][12] = {};
    for (int d0 = 0; d0 < 4; d0++)
        for (int av = 0; av < 16; av++)
            for (int u = -15; u <= 15; u++) {
                const int au = u < 0 ? -u : u;
                if (av != 0 && au > prm.umax[av]) continue;  // IC_Angle's circular patch, cc:70-102
                const int byte = d0 + u + 15;
                icm[d0][av][byte >> 2] |= 1u << (8 * (byte & 3));
                icw[d0][av][byte >> 2] |= (uint32_t)(u + 15) << (8 * (byte & 3));
            }
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_icm), icm, sizeof(icm));
    if (e != hipSuccess) return e;
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_icw), icw, sizeof(icw));
    if (e != hipSuccess) return e;
    return hipMemcpyToSymbol(HIP_SYMBOL(c_umax), prm.umax, sizeof(prm.umax));
}

// Orders this lane's LDS accesses against the other lanes of its wave.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// XCD-aware workgroup -> (frame, block) map for 1-D grids of nframes * per_frame
// workgroups.  The dispatcher hands consecutive workgroup ids to the 8 XCDs round robin
// and each XCD has its own L2; with nframes % 8 == 0, XCD x runs whole frames x, x+8,
// ... in block order, so the halos / patches that neighbouring blocks of a frame share
// are fetched into one L2 once, and every kernel of the pipeline keeps frame f on the
// same XCD (its L2 may still hold what the previous kernel wrote).
constexpr int kXcds = 8;
__device__ __forceinline__ void xcd_frame_block(int per_frame, int nframes, int& f, int& blk) {
    const int lin = blockIdx.x;
    if (nframes % kXcds != 0) {
        f = lin / per_frame;
        blk = lin - f * per_frame;
        return;
    }
    const int x = lin % kXcds, k = lin / kXcds;
    const int fl = k / per_frame;
    blk = k - fl * per_frame;
    f = fl * kXcds + x;
}

// ------------------------------------------------------------------ pyramid

typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));

#ifndef ORBX_PZ_QWORD
#define ORBX_PZ_QWORD 0  // 1: k_pyramid<true> reads a source row window as two qword LDS reads (r05b: slower)
#endif

// 24 x 24 -> high 32 bits of the 48-bit product (v_mul_hi_u32_u24)
__device__ __forceinline__ uint32_t mulhi24(uint32_t a, uint32_t b) {
    return (uint32_t)(((unsigned long long)(a & 0xffffff) * (b & 0xffffff)) >> 32);
}

// The whole pyramid of one tile per workgroup (ORBextractor::ComputePyramid,
// ORBextractor.cc:1635-1694): level 0 is the input frame (cc:1688-1690; the
// REFLECT_101 border is never read by extraction), level l is
// cv::resize(level l-1 ROI, INTER_LINEAR) (cc:1656-1661), OpenCV 3.3.1 fixed point:
// h = S[sx0]*a0 + S[sx1]*a1 (exact), dst = ((b0*(h0>>4))>>16 + (b1*(h1>>4))>>16 + 2)>>2.
// The tile's needed rectangle of every level (its own pixels plus the source footprint
// of the next level, orbx_geometry.h) lives in LDS, ping-ponging between two buffers,
// so the L-level cascade is one launch: only level 0 is read from HBM, and every
// pixel a tile owns is written once.  Threads own a column quad and a run of rows;
// each source row's horizontal sums are computed once and reused by the (one or two)
// output rows that read it.  (b*(h>>4))>>16 is one v_mul_hi_u32_u24 on (b<<8, (h>>4)<<8).
// Write the bytes of quad [x, x+4) that fall in the owned columns [ox0, ox1).
__device__ __forceinline__ void store_owned_quad(uint8_t* o, int x, int ox0, int ox1, uint32_t packed) {
    if (x >= ox0 && x + 4 <= ox1) {
        *(uint32_t*)o = packed;
    } else {
#pragma unroll
        for (int b = 0; b < 4; b++)
            if (x + b >= ox0 && x + b < ox1) o[b] = (uint8_t)(packed >> (8 * b));
    }
}

// Thread -> (column quad, row group) split of a level rectangle nq quads wide: G groups
// of nqp lanes; the quotient comes from a float reciprocal (exact for tid < 256).
struct QuadSplit {
    int nqp, G, q, gr;
};
__device__ __forceinline__ QuadSplit quad_split(int nq, int tid) {
    QuadSplit s;
    s.nqp = min(nq, 256);
    s.G = 256 / s.nqp;
    s.gr = (int)(((float)tid + 0.5f) * (1.0f / (float)s.nqp));
    s.q = tid - s.gr * s.nqp;
    return s;
}

#ifdef ORBX_PZ_WAVES
#define ORBX_PZ_ATTR __attribute__((amdgpu_waves_per_eu(ORBX_PZ_WAVES)))
#else
#define ORBX_PZ_ATTR
#endif
template <bool WIN>
__global__ __launch_bounds__(256) ORBX_PZ_ATTR void k_pyramid(const uint8_t* __restrict__ src, size_t frame_pitch, size_t stride,
                                                 int vec4, uint8_t* __restrict__ pyr, long long fb,
                                                 const LevelGeom* __restrict__ lv, int L,
                                                 const int16_t* __restrict__ rtab, int pz_off, int tiles_pf,
                                                 int nframes, int lds_a, int* __restrict__ status, int l0_store) {
    extern __shared__ __align__(16) uint8_t s_pz[];
    int f, tile;
    xcd_frame_block(tiles_pf, nframes, f, tile);
    const int tid = threadIdx.x;
    // the frame's status word starts clean here (k_octree ORs into it later on this stream):
    // no separate memset launch ahead of every extraction
    if (tile == 0 && tid == 0) status[f] = 0;
    const int16_t* R = rtab + pz_off + (size_t)tile * L * 8;
    uint8_t* const frame = pyr + (size_t)f * fb;
    // LDS rows of a level hold its needed columns widened to whole quads, [x0 & ~3, ...)
    // ---- level 0: load the needed rectangle into buffer A, write the owned part
    {
        const int x0 = R[0], y0 = R[1], x1 = R[2], y1 = R[3];
        const int ox0 = R[4], oy0 = R[5], ox1 = R[6], oy1 = R[7];
        const LevelGeom& g = lv[0];
        if (x1 > x0 && y1 > y0) {
            const int xa = x0 & ~3;
            const int nq = (x1 - xa + 3) >> 2, hn = y1 - y0, ostride = 4 * nq;
            const QuadSplit sp = quad_split(nq, tid);
            const uint8_t* in = src + (size_t)f * frame_pitch;
            if (sp.gr < sp.G) {
                for (int qq = sp.q; qq < nq; qq += sp.nqp) {
                    const int x = xa + 4 * qq;
                    const bool full = x + 4 <= g.w;
                    const bool own_x = x + 4 > ox0 && x < ox1;
                    for (int r0 = sp.gr; r0 < hn; r0 += 8 * sp.G) {  // 8 rows in flight
                        uint32_t v[8];
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            const int y = y0 + min(r0 + k * sp.G, hn - 1);
                            const uint8_t* p = in + (size_t)y * stride + x;
                            if (vec4 && full) {
                                v[k] = *(const uint32_t*)p;
                            } else if (x >= 4 && x + 8 <= g.w) {
                                // an unaligned row (e.g. 1241-byte KITTI rows): the two aligned
                                // dwords around the quad, funnel-shifted; both lie inside the
                                // row (from x - 3 >= 1 to x + 7 < w), so the row's first quad
                                // takes the byte loop below and nothing before the caller's
                                // first row is read
                                // (pointer arithmetic, not an integer round trip: the loads
                                // stay global, not flat)
                                const int sh = (int)((uintptr_t)p & 3);
                                const uint32_t* q = (const uint32_t*)(p - sh);
                                const uint32_t lo = q[0], hi = q[sh ? 1 : 0];
                                v[k] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
                            } else {
                                uint32_t w = 0;
                                for (int b = 0; b < 4 && x + b < g.w; b++) w |= (uint32_t)p[b] << (8 * b);
                                v[k] = w;
                            }
                        }
#pragma unroll
                        for (int k = 0; k < 8; k++) {
                            const int r = r0 + k * sp.G;
                            if (r < hn) {
                                *(uint32_t*)&s_pz[r * ostride + 4 * qq] = v[k];
                                const int y = y0 + r;
                                // l0_store 0: level 0 is read in place from the input by the
                                // later stages (orbx_extractor_set_level0_in_place)
                                if (l0_store && own_x && y >= oy0 && y < oy1)
                                    store_owned_quad(frame + g.off + (size_t)y * g.pitch + x, x, ox0, ox1, v[k]);
                            }
                        }
                    }
                }
            }
        }
    }
    // ---- levels 1..L-1 from the previous level's rectangle in LDS.
    // h = S[sx0]*a0 + S[sx1]*a1 is kept as hm = h & ~15 and the vertical step
    // (b*(h>>4))>>16 = (b*hm)>>20 is one v_mul_hi_u32_u24 of (b << 12, hm).  The result
    // needs no saturation: a0 + a1 <= 2049 and b0 + b1 <= 2049 bound it by 255.
    for (int l = 1; l < L; l++) {
        const int16_t* Rp = R + 8 * (l - 1);
        const int16_t* Rl = R + 8 * l;
        const int sxa = Rp[0] & ~3, sy0 = Rp[1], sstride = 4 * ((Rp[2] - sxa + 3) >> 2);
        const int x0 = Rl[0], y0 = Rl[1], x1 = Rl[2], y1 = Rl[3];
        const int ox0 = Rl[4], oy0 = Rl[5], ox1 = Rl[6], oy1 = Rl[7];
        const LevelGeom& g = lv[l];
        const int16_t* xt = rtab + g.xtab_off;
        const int xa = x0 & ~3;
        const int nq = (x1 - xa + 3) >> 2, hn = y1 - y0, ostride = 4 * nq;
        const QuadSplit sp = quad_split(nq, tid);
        const int rc = (hn + sp.G - 1) / sp.G;
        const int ra = sp.gr * rc, rb = min(hn, ra + rc);
        const bool act = x1 > x0 && y1 > y0 && sp.gr < sp.G && ra < rb;
        // the first quad's column taps (sx0, sx1, a0, a1 as 4 x int16) and the first 8
        // rows' taps are loaded before the barrier: their latency hides in the wait for
        // the previous level.  Columns outside [x0, x1) (quad widening) borrow the nearest
        // column's taps (the quad's source span stays monotone): their bytes are computed
        // but never read by the next level and never owned.
        const int16_t* yt = rtab + g.ytab_off + 4 * (y0 + ra);
        int2 xtp[4], yv[8];  // rtab is padded at the end: 8 rows' taps are always readable
        if (act) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int x = xa + 4 * sp.q + k;
                xtp[k] = *(const int2*)(xt + 4 * min(max(x, x0), x1 - 1));
            }
#pragma unroll
            for (int k = 0; k < 8; k++) yv[k] = *(const int2*)(yt + 4 * k);
        }
        __syncthreads();
        if (!act) continue;
        const uint8_t* sb = s_pz + ((l & 1) ? 0 : lds_a);
        uint8_t* ob = s_pz + ((l & 1) ? lds_a : 0);
        // owned rows of this thread's run, relative to the rectangle
        const int wlo = max(ra, oy0 - y0), whi = min(rb, oy1 - y0);
        for (int qq = sp.q; qq < nq; qq += sp.nqp) {
            const int x = xa + 4 * qq;
            // 0: not owned, 1: whole quad owned, 2: partly owned
            const int own = (x + 4 <= ox0 || x >= ox1) ? 0 : ((x >= ox0 && x + 4 <= ox1) ? 1 : 2);
            if (qq != sp.q) {  // a second quad (rectangles over 1024 columns): reload
#pragma unroll
                for (int k = 0; k < 4; k++) xtp[k] = *(const int2*)(xt + 4 * min(max(x + k, x0), x1 - 1));
#pragma unroll
                for (int k = 0; k < 8; k++) yv[k] = *(const int2*)(yt + 4 * k);
            }
            int c0[4], c1[4];
            uint32_t a0[4], a1[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                c0[k] = (int16_t)(xtp[k].x & 0xffff) - sxa;
                c1[k] = (int16_t)(xtp[k].x >> 16) - sxa;
                a0[k] = (uint32_t)(xtp[k].y & 0xffff);
                a1[k] = (uint32_t)xtp[k].y >> 16;
            }
            // WIN (the plan checked that every quad's source bytes c0[0] .. c1[3] span at
            // most 8): the row's bytes come from three aligned dwords, shifted to start
            // at c0[0] (two v_alignbyte); then per column one v_perm_b32 pairs bytes c0,
            // c1 as u16 halves and one v_dot2_u32_u16 with (a0, a1) gives h.
            const int wbase = c0[0] & ~3, wsh = c0[0] & 3;
            uint32_t wsel[4];
            ushort2_t wab[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                wsel[k] = (uint32_t)(c0[k] - c0[0]) | 0x0c00u | ((uint32_t)(c1[k] - c0[0]) << 16) | 0x0c000000u;
                wab[k] = ushort2_t{(unsigned short)a0[k], (unsigned short)a1[k]};
            }
            const int16_t* yp = yt;
            uint8_t* lp = ob + ra * ostride + 4 * qq;
            uint8_t* gp = frame + g.off + (size_t)(y0 + ra) * g.pitch + x;
            int s_cur = -1;
            const uint8_t* srow = sb;
            uint32_t hc[4] = {0, 0, 0, 0}, hp[4] = {0, 0, 0, 0};
            for (int rr = ra; rr < rb; rr += 8) {
                if (rr != ra) {  // the next 8 rows' taps
#pragma unroll
                    for (int k = 0; k < 8; k++) yv[k] = *(const int2*)(yp + 4 * k);
                }
                yp += 32;
#pragma unroll
                for (int kb = 0; kb < 8; kb++) {
                    const int r = rr + kb;
                    if (r >= rb) break;
                    const int2 t = yv[kb];
                    const int r0 = (int16_t)(t.x & 0xffff), r1 = (int16_t)(t.x >> 16);
                    while (s_cur < r1) {  // the source rows are monotone; each is summed once
                        if (s_cur < 0) {
                            s_cur = r0;
                            srow = sb + (r0 - sy0) * sstride;
                        } else {
                            s_cur++;
                            srow += sstride;
                        }
                        if constexpr (WIN) {
#if ORBX_PZ_QWORD
                            // two 8-byte aligned qword reads: a wave's 32-lane group then
                            // spans ~19 qwords over LDS's 64 dword banks (conflict-free),
                            // where three dword reads spread ~38 dwords over 32 banks
                            // (pointer arithmetic only: an integer round trip would turn the
                            // reads into flat loads)
                            const uint8_t* pw = srow + wbase + wsh;
                            const int mis = (int)((uintptr_t)pw & 7);
                            const uint2* qp = (const uint2*)(pw - mis);
                            const uint2 qa = qp[0];
                            asm volatile("" ::: "memory");  // two ds_read_b64, not one ds_read2_b64 (8 cycles)
                            const uint2 qb = qp[1];
                            const bool hi4 = (mis & 4) != 0;
                            const uint32_t e0 = hi4 ? qa.y : qa.x, e1 = hi4 ? qb.x : qa.y, e2 = hi4 ? qb.y : qb.x;
                            const uint32_t lo = __builtin_amdgcn_alignbyte(e1, e0, (uint32_t)mis & 3);
                            const uint32_t hi = __builtin_amdgcn_alignbyte(e2, e1, (uint32_t)mis & 3);
#else
                            const uint32_t* wp = (const uint32_t*)(srow + wbase);
                            const uint32_t d0 = wp[0], d1 = wp[1], d2 = wp[2];
                            const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, wsh);
                            const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, wsh);
#endif
#pragma unroll
                            for (int k = 0; k < 4; k++) {
                                hp[k] = hc[k];
                                const uint32_t pr = __builtin_amdgcn_perm(hi, lo, wsel[k]);
                                hc[k] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, pr), wab[k], 0u, false) &
                                        ~15u;
                            }
                        } else {
#pragma unroll
                            for (int k = 0; k < 4; k++) {
                                hp[k] = hc[k];
                                // two byte reads (a merged u16 read would be unaligned)
                                hc[k] = (srow[c0[k]] * a0[k] + srow[c1[k]] * a1[k]) & ~15u;
                            }
                        }
                    }
                    const uint32_t b0 = ((uint32_t)t.y & 0xffffu) << 12, b1 = ((uint32_t)t.y >> 16) << 12;
                    const bool same = r0 == s_cur;
                    uint32_t packed = 0;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t v = (mulhi24(b0, same ? hc[k] : hp[k]) + mulhi24(b1, hc[k]) + 2) >> 2;
                        packed |= v << (8 * k);
                    }
                    *(uint32_t*)lp = packed;
                    if (own != 0 && r >= wlo && r < whi) {
                        if (own == 1) *(uint32_t*)gp = packed;
                        else
                            store_owned_quad(gp, x, ox0, ox1, packed);
                    }
                    lp += ostride;
                    gp += g.pitch;
                }
            }
        }
    }
}

// ------------------------------------------------------------------ FAST score + blur

typedef short short2_t __attribute__((ext_vector_type(2)));

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

// FAST-9/16 corner strength M = max over the 16 contiguous 9-arcs of
// max(min(v - ring), min(ring - v)).  At threshold t the pixel is a corner iff
// M > t, and cornerScore<16> then returns max(t, M) - 1 = M - 1, independent of t
// (features2d/fast.cpp FAST_t / fast_score.cpp cornerScore<16>).  Both signs are
// evaluated at once in packed pairs (x, 255 - x): per arc, min(x - v) = min(x) - v and
// min(v - x) = min(255 - x) - (255 - v), so the arc minima of the pairs are taken first
// and (v, 255 - v) is subtracted once.  The pairs are f16 1024 + (x, 255 - x): f16 bits
// 0x6400 + n for n < 1024, i.e. one v_mad_i32_i24 per ring pixel, x * (1 - 2^16) +
// 0x64FF6400, and every value stays an exact small integer.  That admits gfx950's
// 3-input v_pk_minimum3_f16 / v_pk_maximum3_f16: windows of 3 (16), arcs of 9 as
// three windows of 3 (16), the maximum over the arcs (8) -- 40 packed operations.
__device__ __forceinline__ int fast_strength(const uint8_t* c, int pitch) {
    const int off[16] = {0 + 3 * pitch,  1 + 3 * pitch,  2 + 2 * pitch,  3 + 1 * pitch,
                         3,              3 - 1 * pitch,  2 - 2 * pitch,  1 - 3 * pitch,
                         0 - 3 * pitch, -1 - 3 * pitch, -2 - 2 * pitch, -3 - 1 * pitch,
                         -3,            -3 + 1 * pitch, -2 + 2 * pitch, -1 + 3 * pitch};
    const int v = c[0];
    half2_t d[16];
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = __builtin_bit_cast(half2_t, (int)c[off[k]] * -65535 + 0x64ff6400);
    auto mn3 = [](half2_t a, half2_t b, half2_t e) {
        return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), e);
    };
    auto mx3 = [](half2_t a, half2_t b, half2_t e) {
        return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), e);
    };
    half2_t t3[16], arc[16];
#pragma unroll
    for (int j = 0; j < 16; j++) t3[j] = mn3(d[j], d[(j + 1) & 15], d[(j + 2) & 15]);
#pragma unroll
    for (int j = 0; j < 16; j++) arc[j] = mn3(t3[j], t3[(j + 3) & 15], t3[(j + 6) & 15]);
    const half2_t b0 = mx3(arc[0], arc[1], arc[2]), b1 = mx3(arc[3], arc[4], arc[5]);
    const half2_t b2 = mx3(arc[6], arc[7], arc[8]), b3 = mx3(arc[9], arc[10], arc[11]);
    const half2_t b4 = mx3(arc[12], arc[13], arc[14]);
    const half2_t best = __builtin_elementwise_maximum(mx3(b0, b1, b2), mx3(b3, b4, arc[15]));
    // (min x - v, v - max x), exact in f16
    const half2_t r = best - __builtin_bit_cast(half2_t, v * -65535 + 0x64ff6400);
    const _Float16 M = __builtin_elementwise_maximum(__builtin_elementwise_maximum(r.x, r.y), (_Float16)0);
    return (unsigned short)M;  // v_max3_f16 + v_cvt_u16_f16
}

__device__ __forceinline__ int reflect101(int i, int n) {
    i = i < 0 ? -i : i;
    return i >= n ? 2 * n - 2 - i : i;
}

constexpr int kTW = kLtTW, kTH = kLtTH;  // level tile (outputs) of k_level_tiles
static_assert(kTW == 64 && kTH % 16 == 0, "k_level_tiles maps 16 column quads x kTH rows");
#ifndef ORBX_LT_LOAD
#define ORBX_LT_LOAD 16  // k_level_tiles staging load width in bytes (4 or 16)
#endif
constexpr int kLU = ORBX_LT_LOAD;  // staged row: image columns X0-kSX .. X0+63+kSX
constexpr int kSX = kLU == 16 ? 16 : 4;
// row pitch: 16-byte loads stage 96 columns + 8 pad bytes (26 dwords: rows r and r + 16
// share a bank of ds_read_b32's 32; 24 dwords would put rows r and r + 4 together)
constexpr int kSW = kLU == 16 ? kTW + 2 * kSX + 8 : kTW + 2 * kSX;
static_assert(kLU == 4 || kLU == 16, "staging load width");
typedef std::conditional_t<kLU == 16, uint4, uint32_t> lt_load_t;


// Bytes [c+dx, c+dx+3] of a row from its aligned dwords at c-4 (lo), c (mid), c+4 (hi),
// dx in [-4, 4].
__device__ __forceinline__ uint32_t row_bytes(uint32_t lo, uint32_t mid, uint32_t hi, int dx) {
    return dx == -4 ? lo
                    : dx < 0 ? __builtin_amdgcn_alignbyte(mid, lo, 4 + dx)
                             : (dx == 0 ? mid : (dx == 4 ? hi : __builtin_amdgcn_alignbyte(hi, mid, dx)));
}

// Horizontal 7-tap blur sums (exact, <= 257 * 255) of 4 consecutive pixels as two
// v_dot4_u32_u8 per pixel: taps 18,34,49,55 on bytes x-3..x, taps 49,34,18 on x+1..x+3.
__device__ __forceinline__ void blur_row4(uint32_t lo, uint32_t mid, uint32_t hi, uint32_t out[4]) {
    constexpr uint32_t kW1 = 18u | (34u << 8) | (49u << 16) | (55u << 24);
    constexpr uint32_t kW2 = 49u | (34u << 8) | (18u << 16);
#pragma unroll
    for (int j = 0; j < 4; j++)
        out[j] = __builtin_amdgcn_udot4(row_bytes(lo, mid, hi, j - 3), kW1,
                                        __builtin_amdgcn_udot4(row_bytes(lo, mid, hi, j + 1), kW2, 0u, false), false);
}
// bytes 0,1 / 2,3 of a dword zero-extended into the two 16-bit halves
__device__ __forceinline__ uint32_t lo_pair(uint32_t d) { return __builtin_amdgcn_perm(0u, d, 0x0c010c00u); }
__device__ __forceinline__ uint32_t hi_pair(uint32_t d) { return __builtin_amdgcn_perm(0u, d, 0x0c030c02u); }

// Inclusive prefix sum over the 64 lanes of a wave (all lanes active): DPP row_shr
// 1/2/4/8 inside each 16-lane row, then row_bcast:15 and row_bcast:31 across rows.
__device__ __forceinline__ uint32_t wave_inclusive_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}

// One 64x48 tile of one pyramid level per workgroup, all levels and frames in one
// launch (XCD-aware frame placement).  The tile plus a 3-pixel REFLECT_101 margin is
// staged in LDS once and feeds both per-pixel products of the level:
//  * GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) of the level ROI clone
//    (ORBextractor.cc:1587-1595), OpenCV 3.3.1 8U fixed point: taps
//    {18,34,49,55,49,34,18}, exact integer rows (<= 257*255, fits u16, packed
//    v_pk_mad_u16 on 4 pixels per lane), column (sum + 2^15) >> 16, saturate;
//  * the FAST strength map M on the FAST detection area [19, w-19) x [19, h-19).
//    Only M > t_q (t_q = min(iniThFAST, minThFAST)) can ever make a keypoint or a
//    non-zero NMS neighbour in k_fast_cells, and M > t requires two adjacent compass
//    points (ring 0/4/8/12) beyond t on the same side (every 9-arc holds two).  So
//    a cheap 4-pixels-per-lane compass test rejects most pixels (M := 0), the
//    survivors are compacted and only they run the full 16-arc strength.
__global__ __launch_bounds__(256) void k_level_tiles(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                                     uint8_t* __restrict__ score, long long fb,
                                                     const LevelGeom* __restrict__ lv, int L, int tiles_pf,
                                                     int nframes, int tq, const uint8_t* __restrict__ l0,
                                                     long long l0_fp, int l0_pitch) {
    __shared__ __align__(16) uint8_t s_in[kTH + 6][kSW];
    __shared__ __align__(16) uint8_t s_m[kTH][kTW];
    // the survivor list (+ per-lane dump slots for branch-free appends) and, after the
    // strength pass, the blur row sums as (row 2p, row 2p+1) u16 pairs share one buffer
    constexpr int kListB = (kTH * kTW + 128) * 2, kRowpB = (kTH + 6) / 2 * kTW * 4;
#ifndef ORBX_LT_LDS_PAD
#define ORBX_LT_LDS_PAD 0
#endif
    __shared__ __align__(16) uint8_t s_u[(kListB > kRowpB ? kListB : kRowpB) + ORBX_LT_LDS_PAD];
    uint16_t* const s_list = (uint16_t*)s_u;
    uint32_t (*const s_rowp)[kTW] = (uint32_t (*)[kTW])s_u;
    __shared__ int s_n;
    int f, tile;
    xcd_frame_block(tiles_pf, nframes, f, tile);
    const int tid = threadIdx.x, lane = tid & 63;
    int l = 0;
    while (l + 1 < L && tile >= lv[l + 1].tile_first) l++;
    const LevelGeom& g = lv[l];
    const int t = tile - g.tile_first;
    const int ty = t / g.tiles_x;
    const int X0 = (t - ty * g.tiles_x) * kTW, Y0 = ty * kTH;
    // level 0 from the input frame itself when it is read in place (l0 != null)
    const bool in0 = l == 0 && l0 != nullptr;
    const uint8_t* img = in0 ? l0 + (size_t)f * l0_fp : pyr + (size_t)f * fb + g.off;
    const int ipitch = in0 ? l0_pitch : g.pitch;
    // ---- stage rows Y0-3 .. Y0+kTH+2, columns X0-16 .. X0+79 (REFLECT_101 at the ROI
    // edges) as 16-byte loads (pitch and level offsets are multiples of 64); all loads
    // of a thread are issued before the LDS stores: no per-load round trip
    {
        constexpr int kRow = (kTW + 2 * kSX) / kLU, kN = (kTH + 6) * kRow, kPer = (kN + 255) / 256;
        const bool edge = !(X0 >= kSX && X0 + kTW + kSX <= g.w);
        lt_load_t v[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int i = min(tid + 256 * k, kN - 1);
            const int r = i / kRow, cu = i - r * kRow;
            // edge tile: the start column clamped into the row (a load holding an in-range
            // column never clamps: X0 and pitch are multiples of 64)
            const int col = edge ? min(max(X0 - kSX + kLU * cu, 0), ipitch - kLU) : X0 - kSX + kLU * cu;
            v[k] = *(const lt_load_t*)(img + (size_t)reflect101(Y0 + r - 3, g.h) * ipitch + col);
        }
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int i = tid + 256 * k;
            const int r = i / kRow, cu = i - r * kRow;
            if (i < kN) *(lt_load_t*)&s_in[r][kLU * cu] = v[k];
        }
        if (edge) {
            // the only reflected columns anything reads, -3..-1 and w..w+2 (the blur's
            // reach; FAST stays inside [16, w - 16)), are rewritten from the staged row
            __syncthreads();
            for (int i = tid; i < (kTH + 6) * 6; i += 256) {
                const int r = i / 6, k = i - 6 * r;
                const int col = k < 3 ? -1 - k : g.w + k - 3;  // REFLECT_101 source: -col or 2w - 2 - col
                const int sc = col - X0 + kSX, ss = (k < 3 ? -col : 2 * g.w - 2 - col) - X0 + kSX;
                if (sc >= 0 && sc < kSW) s_in[r][sc] = s_in[r][ss];
            }
        }
    }
    if (tid == 0) s_n = 0;
    for (int i = tid; i < kTH * kTW / 4; i += 256) ((uint32_t*)s_m)[i] = 0u;
    __syncthreads();
    // ---- FAST compass test on the detection area, compaction of the survivors.
    // A thread always owns columns 4j..4j+3 (j = tid & 15) of rows tid/16 + 16 i, so
    // its detection-area column mask is computed once.
    {
        const int j = tid & 15, c0 = kSX + 4 * j, x0 = X0 + 4 * j;
        unsigned colmask = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) colmask |= (x0 + k >= kEdge && x0 + k < g.w - kEdge) ? 1u << k : 0u;
        const short2_t tq1 = {(short)(tq + 1), (short)(tq + 1)};
        unsigned pass = 0;  // bit 4 it + k: pixel (row tid/16 + 16 it, column 4j + k) passes
#pragma unroll
        for (int it = 0; it < kTH / 16; it++) {
            const int r = (tid >> 4) + 16 * it;
            const int y = Y0 + r;
            if (colmask != 0 && y >= kEdge && y < g.h - kEdge) {
                const uint32_t* rc = (const uint32_t*)&s_in[r + 3][c0];
                const uint32_t V = rc[0];
                const uint32_t C0 = *(const uint32_t*)&s_in[r + 6][c0];  // ring 0  (0, +3)
                const uint32_t C8 = *(const uint32_t*)&s_in[r][c0];      // ring 8  (0, -3)
                const uint32_t C4 = row_bytes(rc[-1], rc[0], rc[1], 3);   // ring 4  (+3, 0)
                const uint32_t C12 = row_bytes(rc[-1], rc[0], rc[1], -3); // ring 12 (-3, 0)
                uint32_t q[2];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const short2_t v = __builtin_bit_cast(short2_t, h ? hi_pair(V) : lo_pair(V));
                    const short2_t a0 = __builtin_bit_cast(short2_t, h ? hi_pair(C0) : lo_pair(C0)) - v;
                    const short2_t a4 = __builtin_bit_cast(short2_t, h ? hi_pair(C4) : lo_pair(C4)) - v;
                    const short2_t a8 = __builtin_bit_cast(short2_t, h ? hi_pair(C8) : lo_pair(C8)) - v;
                    const short2_t a12 = __builtin_bit_cast(short2_t, h ? hi_pair(C12) : lo_pair(C12)) - v;
                    // bright: min of an adjacent pair of (x - v); dark: min of (v - x) = -max(x - v)
                    const short2_t br = __builtin_elementwise_max(
                        __builtin_elementwise_max(__builtin_elementwise_min(a0, a4), __builtin_elementwise_min(a4, a8)),
                        __builtin_elementwise_max(__builtin_elementwise_min(a8, a12), __builtin_elementwise_min(a12, a0)));
                    const short2_t dk = __builtin_elementwise_min(
                        __builtin_elementwise_min(__builtin_elementwise_max(a0, a4), __builtin_elementwise_max(a4, a8)),
                        __builtin_elementwise_min(__builtin_elementwise_max(a8, a12), __builtin_elementwise_max(a12, a0)));
                    // max(br, -dk) - (tq + 1) >= 0 <=> the pixel passes; sign in bits 15 / 31
                    q[h] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(br, short2_t{0, 0} - dk) - tq1);
                }
                // sign bytes of the 4 pixels -> bit k (clear sign = pass)
                const uint32_t sb = ~__builtin_amdgcn_perm(q[1], q[0], 0x07050301u) & 0x80808080u;
                pass |= ((((sb >> 7) * 0x01020408u) >> 24) & colmask) << (4 * it);
            }
        }
        // one wave-level append for the thread's kTH/16 x 4 pixels, one LDS atomic per
        // wave.  Inside the wave's block the entries go iteration-major (all row-group-0
        // pixels of the wave, then row group 1, ...): 32 consecutive entries then come
        // from adjacent rows, whose ring bytes the strength loop reads from distinct LDS
        // banks (thread-major order put rows r, r + 16, r + 32 -- one bank -- together).
        // Per-iteration counts in 10-bit fields, exclusive offsets from one DPP wave scan.
        static_assert(kTH / 16 <= 3, "three 10-bit count fields");
        uint32_t C = 0;
#pragma unroll
        for (int it = 0; it < kTH / 16; it++) C |= (uint32_t)__popc((pass >> (4 * it)) & 15u) << (10 * it);
        const uint32_t S = wave_inclusive_sum(C);
        const uint32_t T = __builtin_amdgcn_readlane(S, 63), E = S - C;
        int tot = 0;
#pragma unroll
        for (int it = 0; it < kTH / 16; it++) tot += (T >> (10 * it)) & 1023u;
        int base = 0;
        if (lane == 0 && tot) base = atomicAdd(&s_n, tot);
        base = __builtin_amdgcn_readfirstlane(base);
        const int dump = kTH * kTW + 2 * lane;  // per-lane dump slots: no shared address
#pragma unroll
        for (int it = 0; it < kTH / 16; it++) {
            int o = base + ((E >> (10 * it)) & 1023u);
            base += (T >> (10 * it)) & 1023u;
            const int rowc = (((tid >> 4) + 16 * it) << 8) | (4 * j);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const unsigned p = (pass >> (4 * it + k)) & 1u;
                s_list[p ? o : dump] = (uint16_t)(rowc + k);
                o += p;
            }
        }
    }
    __syncthreads();
    // ---- exact strength of the survivors
    const int n = s_n;
    for (int i = tid; i < n; i += 256) {
        const int rc = s_list[i];
        const int r = rc >> 8, c = rc & 255;
        s_m[r][c] = (uint8_t)fast_strength(&s_in[r + 3][c + kSX], kSW);
    }
    __syncthreads();
    // ---- blur rows (into the survivor list's buffer, free now): 2 rows x 4 columns per
    // task (dot4), stored as row-pair u16 dwords
    for (int i = tid; i < ((kTH + 6) / 2) * (kTW / 4); i += 256) {
        const int pr = i >> 4, c0 = kSX + 4 * (i & 15);
        const uint32_t* ra = (const uint32_t*)&s_in[2 * pr][c0];
        const uint32_t* rb = (const uint32_t*)&s_in[2 * pr + 1][c0];
        uint32_t a[4], b[4];
        blur_row4(ra[-1], ra[0], ra[1], a);
        blur_row4(rb[-1], rb[0], rb[1], b);
        *(uint4*)&s_rowp[pr][c0 - kSX] = make_uint4(a[0] | (b[0] << 16), a[1] | (b[1] << 16), a[2] | (b[2] << 16),
                                                  a[3] | (b[3] << 16));
    }
    __syncthreads();
    // ---- blur columns and the strength map -> global, two rows x 4 columns per task:
    // rows 2p and 2p+1 read the same four row-pair dwords (staged rows 2p..2p+7), one
    // v_dot2_u32_u16 per pair, column and row, then (sum + 2^15) >> 16
    uint8_t* bout = blur + (size_t)f * fb + g.off;
    uint8_t* mout = score + (size_t)f * fb + g.off;
    for (int i = tid; i < (kTH / 2) * (kTW / 4); i += 256) {
        const int rp = i >> 4, c = 4 * (i & 15);
        const int r = 2 * rp, y = Y0 + r, x = X0 + c;
        if (y >= g.h || x >= g.w) continue;  // kTH is even: row y + 1 is then out too
        const bool two = y + 1 < g.h;
        uint4 q[4];
#pragma unroll
        for (int k = 0; k < 4; k++) q[k] = *(const uint4*)&s_rowp[rp + k][c];
        const ushort2_t we[4] = {ushort2_t{18, 34}, ushort2_t{49, 55}, ushort2_t{49, 34}, ushort2_t{18, 0}};
        const ushort2_t wo[4] = {ushort2_t{0, 18}, ushort2_t{34, 49}, ushort2_t{55, 49}, ushort2_t{34, 18}};
        unsigned se[4] = {1u << 15, 1u << 15, 1u << 15, 1u << 15};  // + the rounding half
        unsigned so[4] = {1u << 15, 1u << 15, 1u << 15, 1u << 15};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            se[0] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, q[k].x), we[k], se[0], false);
            se[1] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, q[k].y), we[k], se[1], false);
            se[2] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, q[k].z), we[k], se[2], false);
            se[3] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, q[k].w), we[k], se[3], false);
            so[0] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, q[k].x), wo[k], so[0], false);
            so[1] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, q[k].y), wo[k], so[1], false);
            so[2] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, q[k].z), wo[k], so[2], false);
            so[3] = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, q[k].w), wo[k], so[3], false);
        }
        uint32_t pe = 0, po = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const unsigned ve = se[k] >> 16, vo = so[k] >> 16;
            pe |= (ve > 255 ? 255u : ve) << (8 * k);
            po |= (vo > 255 ? 255u : vo) << (8 * k);
        }
        const uint32_t me = *(const uint32_t*)&s_m[r][c], mo = *(const uint32_t*)&s_m[r + 1][c];
        const size_t off = (size_t)y * g.pitch + x;
        if (x + 4 <= g.w) {
            *(uint32_t*)(bout + off) = pe;
            *(uint32_t*)(mout + off) = me;
            if (two) {
                *(uint32_t*)(bout + off + g.pitch) = po;
                *(uint32_t*)(mout + off + g.pitch) = mo;
            }
        } else {
            for (int k = 0; x + k < g.w; k++) {
                bout[off + k] = (uint8_t)(pe >> (8 * k));
                mout[off + k] = (uint8_t)(me >> (8 * k));
                if (two) {
                    bout[off + g.pitch + k] = (uint8_t)(po >> (8 * k));
                    mout[off + g.pitch + k] = (uint8_t)(mo >> (8 * k));
                }
            }
        }
    }
}

// ------------------------------------------------------------------ FAST cells

// One wave per cell.  Reproduces cv::FAST(cell, kps, t, true) for t = iniThFAST and,
// if that leaves the cell empty, t = minThFAST (ORBextractor.cc:1091-1104), from the
// strength map M (corner iff M > t, score M - 1).  FAST_t's non-max suppression over
// the 8-neighbourhood, where neighbours outside the cell's detection window or below
// the threshold score 0, keeps a corner p iff M_p > t, M_p >= 2 and M_p exceeds every
// in-window neighbour's M (a neighbour with M_n >= M_p > t always suppresses; one below
// M_p never does) -- threshold-independent apart from M_p > t.  M is sparse (k_level_tiles
// zeroes M <= min(iniTh, minTh)), so the wave stages the window with a zero frame, lists
// the non-zero pixels in raster order (one ballot per row -- per row pair when the window
// is at most 32 wide), tests only those against their neighbours, and writes the
// survivors of the chosen threshold in the same order.
// Staged window row pitch: 68 bytes (64 + zero frame, an odd dword count), a compile-time
// constant.  Measured alternatives (ORBX_FC_PITCH): 44-100 bytes all slower at configs[4]
// (up to -8 %, r05al / r05am), and a pitch sized to the widest window (36 bytes at 30-px
// cells, 4.4 KB less LDS per workgroup) -6 % there (r05ac).  Passing the pitch at run
// time (as that experiment did) cost configs[1] 1.1 % by itself (r05bh).
#ifndef ORBX_FC_PITCH
#define ORBX_FC_PITCH 68
#endif
constexpr int kFcStride = ORBX_FC_PITCH;
#ifndef ORBX_FC_INFLIGHT
#define ORBX_FC_INFLIGHT 8  // k_fast_cells: row steps of byte loads in flight (r05aw: 4 -2 %,
                            // 16 -10 % at configs[1])
#endif
static_assert(kFcStride % 4 == 0 && kFcStride >= 36, "fast_cells window pitch");

__global__ __launch_bounds__(256) void k_fast_cells(const uint8_t* __restrict__ score, long long fb,
                                                    const CellGeom* __restrict__ cells, int ncells,
                                                    int ini_th, int min_th, uint32_t* __restrict__ slots,
                                                    int slots_pf, int* __restrict__ cell_count, int nframes,
                                                    int max_wr, int max_wc) {
    // per wave: (max_wr + 2) framed rows of M (pitch kFcStride >= max_wc + 2, checked by
    // the launcher), then a candidate list of max_wr*max_wc u16
    extern __shared__ __align__(16) uint8_t s_dyn[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int per_wave = (((max_wr + 2) * kFcStride + 2 * max_wr * max_wc) + 15) & ~15;
    int f, cb;
    xcd_frame_block((ncells + 3) / 4, nframes, f, cb);
    const int ci = cb * 4 + wave;
    if (ci >= ncells) return;  // whole wave exits; no block barriers below
    const CellGeom c = cells[ci];
    const int wr = c.rows - 6, wc = c.cols - 6;  // detection window [3,rows-3) x [3,cols-3)
    int count = 0;
    if (wr > 0 && wc > 0) {
        const int ti = ini_th < 0 ? 0 : (ini_th > 255 ? 255 : ini_th);
        const int tm = min_th < 0 ? 0 : (min_th > 255 ? 255 : min_th);
        const int tc = max(min(ti, tm), 1);  // candidates: M > tc
        const uint8_t* src = score + (size_t)f * fb + c.src_off;
        uint8_t* m = s_dyn + wave * per_wave;  // m[(r + 1) * kFcStride + c + 1] = M(r, c)
        uint16_t* list = (uint16_t*)(s_dyn + wave * per_wave + (max_wr + 2) * kFcStride);
        const unsigned long long below = (1ull << lane) - 1;
        // zero frame: rows -1 and wr, column -1 (column wc is written as 0 below)
        for (int i = lane; i < kFcStride; i += 64) {
            m[i] = 0;
            m[(wr + 1) * kFcStride + i] = 0;
        }
        for (int r = lane; r < wr + 2; r += 64) {  // columns -1 and wc
            m[r * kFcStride] = 0;
            m[r * kFcStride + wc + 1] = 0;
        }
        int n = 0;
        const bool pairs = wc <= 32;
        const int col = pairs ? (lane & 31) : lane;
        const int half = pairs ? (lane >> 5) : 0;
        const int rstep = pairs ? 2 : 1;
        const bool act = col < wc;
        // 8 row steps of loads in flight at a time.  The loads are unconditional: the
        // window ends >= 19 rows above the level's bottom and rows are >= 64 wide, so up
        // to 15 rows / 63 columns past it stay inside the frame's block (and the buffer
        // has slack); the values are masked.  The row part of each offset is wave-uniform
        // (scalar adds to the base), the lane part a 32-bit vector offset.
        const uint32_t loff = (uint32_t)(half * c.pitch + col);
        constexpr int kIF = ORBX_FC_INFLIGHT;  // row steps of loads in flight
        for (int r0 = 0; r0 < wr; r0 += kIF * rstep) {
            int v[kIF];
#pragma unroll
            for (int k = 0; k < kIF; k++) {
                // more than 8 steps: rows clamped to the window (at most one row past it)
                const int rk = kIF > 8 ? min(r0 + k * rstep, wr - 1) : r0 + k * rstep;
                v[k] = src[(uint32_t)(rk * c.pitch) + loff];
            }
#pragma unroll
            for (int k = 0; k < kIF; k++) v[k] = (act && r0 + k * rstep + half < wr) ? v[k] : 0;
#pragma unroll
            for (int k = 0; k < kIF; k++) {
                const int rb = r0 + k * rstep;  // first row of this step (wave-uniform)
                if (rb < wr) {
                    const int r = rb + half;
                    // (a pitch of at least 65 holds every lane's column; a smaller one only
                    // the window and its right frame)
                    if (r < wr && (kFcStride >= 65 || col <= wc)) m[(r + 1) * kFcStride + col + 1] = (uint8_t)v[k];
                    const unsigned long long b = __ballot(v[k] > tc);  // raster order: row rb, then rb+1
                    if ((b >> lane) & 1ull) list[n + __popcll(b & below)] = (uint16_t)((r << 8) | col);
                    n += __popcll(b);
                }
            }
        }
        wave_lds_fence();
        // neighbour test of the candidates (zero frame: no bounds checks), both thresholds
        auto keep_of = [&](int i, int& r, int& cc, int& M) -> bool {
            const int rc = list[i];
            r = rc >> 8;
            cc = rc & 255;
            const uint8_t* p = m + (r + 1) * kFcStride + cc + 1;
            M = p[0];
            const int nb = max(max(max(p[-kFcStride - 1], p[-kFcStride]), max(p[-kFcStride + 1], p[-1])),
                               max(max(p[1], p[kFcStride - 1]), max(p[kFcStride], p[kFcStride + 1])));
            return M > nb;  // M > tc >= 1, so M >= 2
        };
        // the first kFcKeep x 64 candidates' outcomes at both thresholds are kept as
        // wave masks, so the write pass below re-tests only candidates past them
        constexpr int kFcKeep = 4;
        unsigned long long mi[kFcKeep], mm[kFcKeep];
        int cnt_i = 0, cnt_m = 0;
        for (int i0 = 0; i0 < n; i0 += 64) {
            bool ki = false, km = false;
            if (i0 + lane < n) {
                int r, cc, M;
                const bool lm = keep_of(i0 + lane, r, cc, M);
                ki = lm && M > ti;
                km = lm && M > tm;
            }
            const unsigned long long bi = __ballot(ki), bm = __ballot(km);
#pragma unroll
            for (int u = 0; u < kFcKeep; u++)
                if (i0 == 64 * u) { mi[u] = bi; mm[u] = bm; }
            cnt_i += __popcll(bi);
            cnt_m += __popcll(bm);
        }
        const bool use_ini = cnt_i > 0;
        count = use_ini ? cnt_i : cnt_m;
        const int t = use_ini ? ti : tm;
        if (count > 0) {
            uint32_t* out = slots + (size_t)f * slots_pf + c.slot_off;
            int base = 0;
            for (int i0 = 0; i0 < n; i0 += 64) {
                bool keep = false;
                int r = 0, cc = 0, M = 0;
                if (i0 < 64 * kFcKeep) {
                    unsigned long long km = 0;
#pragma unroll
                    for (int u = 0; u < kFcKeep; u++)
                        if (i0 == 64 * u) km = use_ini ? mi[u] : mm[u];
                    keep = (km >> lane) & 1ull;
                    if (keep) {
                        const int rc = list[i0 + lane];
                        r = rc >> 8;
                        cc = rc & 255;
                        M = m[(r + 1) * kFcStride + cc + 1];
                    }
                } else if (i0 + lane < n) {
                    keep = keep_of(i0 + lane, r, cc, M) && M > t;
                }
                const unsigned long long b = __ballot(keep);
                if (keep) {
                    const int xr = c.x0 + 3 + cc - kMinBorder;  // relative to minBorderX
                    const int yr = c.y0 + 3 + r - kMinBorder;
                    out[base + __popcll(b & below)] = (uint32_t)xr | ((uint32_t)yr << 12) | ((uint32_t)(M - 1) << 24);
                }
                base += __popcll(b);
            }
        }
    }
    if (lane == 0) cell_count[(size_t)f * ncells + ci] = count;
}

// ------------------------------------------------------------------ block helpers

// In-place exclusive scan of a[0..n) (non-negative) by a 256-thread block; returns the
// total.  `tmp` holds >= 8 ints of LDS.  All threads must call it, after a barrier that
// makes every thread's writes to a[] visible: each thread sums a contiguous run of
// ceil(n / 256) entries (written by other threads), one DPP wave scan and one barrier
// combine the runs, and each thread rewrites its run: two barriers for any n (the
// octree's node lists reach a few thousand entries).
__device__ int block_exscan(int* a, int n, int* tmp) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (n + 255) >> 8;
    const int b0 = min(tid * per, n), b1 = min(b0 + per, n);
    int s = 0;
    for (int i = b0; i < b1; i++) s += a[i];
    const int incl = (int)wave_inclusive_sum((uint32_t)s);
    if (lane == 63) tmp[wave] = incl;
    __syncthreads();
    int run = incl - s;
    for (int k = 0; k < wave; k++) run += tmp[k];
    const int total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
    for (int i = b0; i < b1; i++) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
    return total;
}

// Two in-place exclusive scans (a[0..n), b[0..n), non-negative) in one pass: the same
// two barriers as one block_exscan.  Totals in ta / tb.  tmp: >= 8 ints.
__device__ void block_exscan2(int* a, int* b, int n, int* tmp, int& ta, int& tb) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (n + 255) >> 8;
    const int b0 = min(tid * per, n), b1 = min(b0 + per, n);
    int sa = 0, sb = 0;
    for (int i = b0; i < b1; i++) {
        sa += a[i];
        sb += b[i];
    }
    const int ia = (int)wave_inclusive_sum((uint32_t)sa), ib = (int)wave_inclusive_sum((uint32_t)sb);
    if (lane == 63) {
        tmp[wave] = ia;
        tmp[4 + wave] = ib;
    }
    __syncthreads();
    int ra = ia - sa, rb = ib - sb;
    for (int k = 0; k < wave; k++) {
        ra += tmp[k];
        rb += tmp[4 + k];
    }
    ta = tmp[0] + tmp[1] + tmp[2] + tmp[3];
    tb = tmp[4] + tmp[5] + tmp[6] + tmp[7];
    for (int i = b0; i < b1; i++) {
        const int va = a[i], vb = b[i];
        a[i] = ra;
        b[i] = rb;
        ra += va;
        rb += vb;
    }
    __syncthreads();
}

__device__ __forceinline__ int key_x(uint32_t k) { return (int)(k & 0xfffu); }
__device__ __forceinline__ int key_y(uint32_t k) { return (int)((k >> 12) & 0xfffu); }
__device__ __forceinline__ int key_resp(uint32_t k) { return (int)(k >> 24); }

// ExtractorNode::DivideNode quadrant (ORBextractor.cc:587-641): halves are
// ceil(width/2), ceil(height/2); n1 UL, n2 UR, n3 BL, n4 BR.
__device__ __forceinline__ int quadrant(int x, int y, int x0, int y0, int x1, int y1) {
    const int mx = x0 + ((x1 - x0 + 1) >> 1);
    const int my = y0 + ((y1 - y0 + 1) >> 1);
    return x < mx ? (y < my ? 0 : 2) : (y < my ? 1 : 3);
}

__device__ __forceinline__ void child_box(int q, int x0, int y0, int x1, int y1, int& cx0, int& cy0,
                                          int& cx1, int& cy1) {
    const int mx = x0 + ((x1 - x0 + 1) >> 1);
    const int my = y0 + ((y1 - y0 + 1) >> 1);
    cx0 = (q & 1) ? mx : x0;
    cx1 = (q & 1) ? x1 : mx;
    cy0 = (q & 2) ? my : y0;
    cy1 = (q & 2) ? y1 : my;
}

// ------------------------------------------------------------------ octree

// Full passes with at most this many nodes count their quadrants per distinct (node,
// quadrant) of a wave (wave_count_q: a readlane / ballot / atomic loop); larger lists use
// one LDS atomic per key.  Until round 5 the loop ran up to 64 nodes; one atomic per key
// measured faster at every size (r05i, interleaved: configs[1] 228.5k -> 229.3-229.7k,
// configs[4] 111.1-111.5k -> 113.4-113.7k frames/s; the single C1 / C3 / C5 call 144 /
// 226 / 234 -> 137 / 206 / 212 us), so 0 turns it off.
#ifndef ORBX_OCT_FEW
#define ORBX_OCT_FEW 0
#endif

// Node list, stored in list order (front first).  Two buffers, swapped every step.
constexpr int kOctKeysReg = 16 * 256;  // keys per level held in registers by k_octree

// atomicAdd(&a[idx], 1) for the active lanes, one atomic per distinct idx of the wave
// (the early octree passes send thousands of keys to a handful of counters).
__device__ __forceinline__ void wave_count(int* a, int idx) {
    const int lane = threadIdx.x & 63;
    unsigned long long act = __ballot(1);
    while (act) {
        const int leader = __ffsll((long long)act) - 1;
        const int t = __builtin_amdgcn_readlane(idx, leader);
        const unsigned long long m = __ballot(idx == t);
        if (lane == leader) atomicAdd(&a[t], __popcll(m));
        act &= ~m;
    }
}

// The same with the four quadrant counters of a node packed as u16 pairs in two words
// (word 2*node + q/2, half q%2): atomicAdd(quadrant q of node nd, 1) per distinct (nd, q).
__device__ __forceinline__ void wave_count_q(uint32_t* a, int idx) {
    const int lane = threadIdx.x & 63;
    unsigned long long act = __ballot(1);
    while (act) {
        const int leader = __ffsll((long long)act) - 1;
        const int t = __builtin_amdgcn_readlane(idx, leader);
        const unsigned long long m = __ballot(idx == t);
        if (lane == leader) atomicAdd(&a[t >> 1], (uint32_t)__popcll(m) << (16 * (t & 1)));
        act &= ~m;
    }
}
__device__ __forceinline__ void add_q(uint32_t* a, int nd, int q) {
    atomicAdd(&a[2 * nd + (q >> 1)], 1u << (16 * (q & 1)));
}
__device__ __forceinline__ int get_q(const uint32_t* a, int nd, int q) {
    return (int)((a[2 * nd + (q >> 1)] >> (16 * (q & 1))) & 0xffffu);
}
// Keys per level the packed counters and keys hold (u16 counts); a level with more
// FAST keypoints is flagged kStatusNodeOverflow.
constexpr int kOctMaxKeys = 65535;
constexpr int kOctStampWords = 16;  // diagnostics row per (frame, level), ORBX_OCT_STAMPS
#ifndef ORBX_OCT_SPLIT_LEVELS
#define ORBX_OCT_SPLIT_LEVELS 1  // batches: the small levels in a second k_octree launch (launch_extract)
#endif
constexpr bool kOctSplitLevels = ORBX_OCT_SPLIT_LEVELS != 0;
#ifndef ORBX_OCT_SPLIT_NUM  // the second launch takes the levels with ncap <= NUM / DEN of level 0's
#define ORBX_OCT_SPLIT_NUM 3
#define ORBX_OCT_SPLIT_DEN 8
#endif
constexpr int kOctNodeBytes = 4 + 8 + 8 + 4 + 2 + 4 + 16 + 2;  // best, ccnt, sa+sb, cnt x2 (u16), sc, crank x2, boxes, inV

struct NodeBuf {
    int16_t *x0, *y0, *x1, *y1;
    uint16_t* cnt;  // keys in the node (<= kOctMaxKeys)
    int16_t* crank;  // creation rank within the step that created the node (< NC)
    uint8_t* inV;   // member of vSizeAndPointerToNode (created last step with >1 key)
};

// One workgroup per (level, frame): gathers the level's FAST keypoints in cell order
// and runs ORBextractor::DistributeOctTree (ORBextractor.cc:667-1013) as a sequence of
// data-parallel list rewrites that reproduce the std::list order exactly:
//  * a full pass (cc:779-862) splits every node with >1 key; children are pushed to
//    the front, so the new list is [children of the last split node (n4..n1), ...,
//    children of the first split node, then the surviving single-key nodes in order];
//  * the final phase (cc:888-971) splits vSizeAndPointerToNode sorted by (size, node
//    address) from the back until the list holds N nodes.  Node addresses are taken
//    in allocation order (hazard H1), i.e. ties go to the later-created
//    node first;
//  * each surviving node keeps its max-response key, first (lowest index) on ties
//    (cc:984-1009).
#ifndef ORBX_OCT_WPE
#define ORBX_OCT_WPE 5  // k_octree's register budget: waves per SIMD (5: <= 102 VGPRs)
#endif
__global__ __launch_bounds__(256, ORBX_OCT_WPE) void k_octree(const LevelGeom* __restrict__ lv, int L,
                                                const uint32_t* __restrict__ slots, int slots_pf,
                                                const CellGeom* __restrict__ cells,
                                                const int* __restrict__ cell_count, int ncells_total,
                                                uint32_t* __restrict__ keys, int* __restrict__ key_node,
                                                int keys_pf, uint32_t* __restrict__ kept, int kept_pf,
                                                int* __restrict__ kept_count, int* __restrict__ status,
                                                int NC, int nframes, unsigned long long* __restrict__ stamps,
                                                uint16_t* __restrict__ dt_list, uint32_t* __restrict__ dt_tile,
                                                int tiles_pf, int l_first) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_tmp[8];
    __shared__ int s_scal[16];
    __shared__ int s_off[256];
    __shared__ int s_src[256];
    __shared__ int s_map[kMaxIni];
    __shared__ int s_icnt[kMaxIni];

    // Level-major order (all frames' level l_first first, then the next level, ...): the
    // long distributions start first and the short ones fill in behind them; frames keep
    // their XCD (frame f on XCD f % 8) when nframes % 8 == 0.  A launch covers the levels
    // l_first .. l_first + gridDim.x / nframes - 1.
    int f, l;
    {
        const int lin = blockIdx.x;
        if (nframes % kXcds == 0) {
            const int per = nframes / kXcds, x = lin % kXcds, k = lin / kXcds;
            l = k / per;
            f = (k - l * per) * kXcds + x;
        } else {
            l = lin / nframes;
            f = lin - l * nframes;
        }
        l += l_first;
    }
    const int tid = threadIdx.x;
    unsigned long long* st = stamps ? stamps + kOctStampWords * ((size_t)f * L + l) : nullptr;
    if (st && tid == 0) {
        st[0] = wall_clock64();
        st[8] = 0;  // final phase: ticks spent ranking vPrev
    }
    const int lane = tid & 63, wave = tid >> 6;
    const LevelGeom& g = lv[l];
    const int N = g.N;

    // LDS carve-up (NC nodes, kOctNodeBytes = 48 B each: at configs[4]'s NC = 960 three
    // workgroups fit a CU).  best: the final phase's (size << 16 | creation rank) keys,
    // then each node's (response << 24 | ~key index) maximum; ccnt: four u16 quadrant
    // counters per node, reused for the children's positions; sc: per-node ne / ranks.
    uint32_t* best = (uint32_t*)smem;                                   // NC
    uint32_t* ccnt = best + NC;                                         // 2*NC (must follow best)
    uint16_t* cpos = (uint16_t*)ccnt;                                   // [4*NC] child positions
    int* sa = (int*)(ccnt + 2 * NC);                                    // NC
    int* sb = sa + NC;                                                  // NC
    uint16_t* cntb = (uint16_t*)(sb + NC);                              // 2*NC
    int16_t* sc = (int16_t*)(cntb + 2 * NC);                            // NC
    int16_t* crkb = sc + NC;                                            // 2*NC
    int16_t* boxb = crkb + 2 * NC;                                      // 8*NC
    uint8_t* inVb = (uint8_t*)(boxb + 8 * NC);                          // 2*NC
    NodeBuf nb0, nb1;
    nb0.x0 = boxb;
    nb0.y0 = boxb + NC;
    nb0.x1 = boxb + 2 * NC;
    nb0.y1 = boxb + 3 * NC;
    nb0.cnt = cntb;
    nb0.crank = crkb;
    nb0.inV = inVb;
    nb1.x0 = boxb + 4 * NC;
    nb1.y0 = boxb + 5 * NC;
    nb1.x1 = boxb + 6 * NC;
    nb1.y1 = boxb + 7 * NC;
    nb1.cnt = cntb + NC;
    nb1.crank = crkb + NC;
    nb1.inV = inVb + NC;

    uint32_t* K = keys + (size_t)f * keys_pf + g.key_off;
    int* KN = key_node + (size_t)f * keys_pf + g.key_off;

    // ---- 1. gather candidates in cell order (vToDistributeKeys, cc:1054-1122)
    // 256 cells at a time: offsets by a block scan, then the chunk's keys are copied
    // flat (key t of the chunk finds its cell by binary search over the offsets), so
    // every thread has several independent loads in flight.
    int n = 0;
    const uint32_t* fslots = slots + (size_t)f * slots_pf;
    for (int cb = 0; cb < g.ncells; cb += 256) {
        const int nc = g.ncells - cb < 256 ? g.ncells - cb : 256;
        if (tid < nc) {
            s_off[tid] = cell_count[(size_t)f * ncells_total + g.cell_first + cb + tid];
            s_src[tid] = cells[g.cell_first + cb + tid].slot_off;
        }
        __syncthreads();
        const int tot = block_exscan(s_off, nc, s_tmp);
        for (int t0 = 0; t0 < tot; t0 += 4 * 256) {
            uint32_t v[4];
            int dst[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int t = t0 + u * 256 + tid;
                int lo = 0, hi = nc - 1;  // last cell with s_off <= t
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (s_off[mid] <= t) lo = mid;
                    else hi = mid - 1;
                }
                const int tc = t < tot ? t : tot - 1;
                dst[u] = t < tot ? n + t : -1;
                v[u] = fslots[s_src[lo] + (tc - s_off[lo])];
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (dst[u] >= 0) K[dst[u]] = v[u];
        }
        n += tot;
        __syncthreads();
    }
    __threadfence_block();
    __syncthreads();
    if (st && tid == 0) {
        st[1] = wall_clock64();
        st[6] = n;
    }
    if (n > kOctMaxKeys) {  // beyond the u16 counters (never on real frames): flagged, not truncated silently
        if (tid == 0) {
            atomicOr(&status[f], kStatusNodeOverflow);
            kept_count[(size_t)f * L + l] = 0;
        }
        if (dt_list)
            for (int t = tid; t < g.tiles_x * g.tiles_y; t += 256) dt_tile[(size_t)f * tiles_pf + g.tile_first + t] = 0u;
        return;
    }

    // The per-key state (packed key, node) of key k lives with thread k % 256 for the
    // whole distribution: in registers when the level has at most kOctKeysReg keys
    // (REG), otherwise in global memory.
    auto tail = [&](auto reg_tag) {
    constexpr bool REG = decltype(reg_tag)::value;
    constexpr int KPT = REG ? kOctKeysReg / 256 : 1;
    uint32_t kr[KPT];
    uint32_t nr[(KPT + 1) / 2];  // node ids (< NC <= 2^15), two per register
    if (REG) {
#pragma unroll
        for (int i = 0; i < KPT; i++) {
            const int k = min(tid + 256 * i, n - 1);
            kr[i] = n > 0 ? K[k] : 0u;
        }
#pragma unroll
        for (int i = 0; i < (KPT + 1) / 2; i++) nr[i] = 0u;
    }
#define FOR_KEYS(BODY)                                                      \
    if (REG) {                                                              \
        _Pragma("unroll") for (int i_ = 0; i_ < KPT; i_++) {                \
            const int k = tid + 256 * i_;                                   \
            if (k < n) {                                                    \
                const uint32_t KK = kr[i_];                                 \
                const int sh_ = 16 * (i_ & 1);                              \
                int NN = (int)((nr[i_ >> 1] >> sh_) & 0xffffu);             \
                BODY                                                        \
                nr[i_ >> 1] = (nr[i_ >> 1] & ~(0xffffu << sh_)) |           \
                              ((uint32_t)NN & 0xffffu) << sh_;             \
            }                                                               \
        }                                                                   \
    } else {                                                                \
        for (int k = tid; k < n; k += 256) {                                \
            const uint32_t KK = K[k];                                       \
            int NN = KN[k];                                                 \
            BODY                                                            \
            KN[k] = NN;                                                     \
        }                                                                   \
    }

    // ---- 2. root nodes (cc:674-742)
    if (tid < g.nIni) s_icnt[tid] = 0;
    __syncthreads();
    FOR_KEYS({
        const int idx = (int)((float)key_x(KK) / g.hX);
        wave_count(s_icnt, idx);
        NN = idx;
    })
    __syncthreads();
    if (tid == 0) {
        int j = 0;
        for (int i = 0; i < g.nIni; i++) {
            if (s_icnt[i] > 0) {
                s_map[i] = j;
                nb0.x0[j] = (int16_t)g.ini_x0[i];
                nb0.x1[j] = (int16_t)g.ini_x0[i + 1];
                nb0.y0[j] = 0;
                nb0.y1[j] = (int16_t)g.height_rel;
                nb0.cnt[j] = (uint16_t)s_icnt[i];
                nb0.crank[j] = i;
                nb0.inV[j] = 0;
                j++;
            } else {
                s_map[i] = -1;
            }
        }
        s_scal[0] = j;  // size
    }
    __syncthreads();
    FOR_KEYS({ NN = s_map[NN]; })
    __syncthreads();

    int cur = 0;
    int size = s_scal[0];
    int guard = 0;
    bool finish = false;
    bool final_phase = false;

    // ---- 3. full passes (cc:758-873)
    while (!finish && !final_phase) {
        if (++guard > 64) { if (tid == 0) atomicOr(&status[f], kStatusIterations); break; }
        const NodeBuf& A = cur ? nb1 : nb0;
        const NodeBuf& B = cur ? nb0 : nb1;
        const int prev = size;
        for (int j = tid; j < size; j += 256) ccnt[2 * j] = ccnt[2 * j + 1] = 0u;
        if (tid == 0) s_scal[1] = 0;
        __syncthreads();
        const bool few = ORBX_OCT_FEW > 0 && size <= ORBX_OCT_FEW;  // (compiled out at 0)
        FOR_KEYS({
            const int nd = NN;
            if (A.cnt[nd] >= 2) {
                const int q = quadrant(key_x(KK), key_y(KK), A.x0[nd], A.y0[nd], A.x1[nd], A.y1[nd]);
                if (few) wave_count_q(ccnt, 4 * nd + q);
                else add_q(ccnt, nd, q);
            }
        })
        __syncthreads();
        int g2 = 0;
        for (int j = tid; j < size; j += 256) {
            const bool split = A.cnt[j] >= 2;
            int ne = 0;
            if (split)
                for (int q = 0; q < 4; q++) {
                    ne += get_q(ccnt, j, q) > 0;
                    g2 += get_q(ccnt, j, q) > 1;
                }
            sa[j] = ne;
            sb[j] = split ? 0 : 1;
            sc[j] = (int16_t)ne;
        }
        if (g2) atomicAdd(&s_scal[1], g2);
        __syncthreads();
        int C, T;
        block_exscan2(sa, sb, size, s_tmp, C, T);
        const int G = s_scal[1];
        const int nsize = C + T;
        if (nsize > NC) { if (tid == 0) atomicOr(&status[f], kStatusNodeOverflow); finish = true; break; }
        for (int j = tid; j < size; j += 256) {
            if (A.cnt[j] >= 2) {
                const int ne = sc[j];
                const int P = C - sa[j] - ne;  // block of the children: sum of ne over later split nodes
                int r = 0;
                for (int q = 0; q < 4; q++) {
                    const int cq = get_q(ccnt, j, q);  // slot q is still a count (earlier slots hold positions)
                    if (cq > 0) {
                        const int pos = P + (ne - 1 - r);  // pushed front in n1..n4 order
                        int cx0, cy0, cx1, cy1;
                        child_box(q, A.x0[j], A.y0[j], A.x1[j], A.y1[j], cx0, cy0, cx1, cy1);
                        B.x0[pos] = (int16_t)cx0;
                        B.y0[pos] = (int16_t)cy0;
                        B.x1[pos] = (int16_t)cx1;
                        B.y1[pos] = (int16_t)cy1;
                        B.cnt[pos] = (uint16_t)cq;
                        B.crank[pos] = (int16_t)(sa[j] + r);
                        B.inV[pos] = cq > 1;
                        cpos[4 * j + q] = (uint16_t)pos;
                        r++;
                    }
                }
            } else {
                const int pos = C + sb[j];
                B.x0[pos] = A.x0[j];
                B.y0[pos] = A.y0[j];
                B.x1[pos] = A.x1[j];
                B.y1[pos] = A.y1[j];
                B.cnt[pos] = A.cnt[j];
                B.crank[pos] = A.crank[j];
                B.inV[pos] = 0;
                sb[j] = pos;
            }
        }
        __syncthreads();
        FOR_KEYS({
            const int nd = NN;
            if (A.cnt[nd] >= 2) {
                const int q = quadrant(key_x(KK), key_y(KK), A.x0[nd], A.y0[nd], A.x1[nd], A.y1[nd]);
                NN = cpos[4 * nd + q];
            } else {
                NN = sb[nd];
            }
        })
        __syncthreads();
        cur ^= 1;
        size = nsize;
        if (size >= N || size == prev)
            finish = true;
        else if (size + G * 3 > N)
            final_phase = true;
    }

    if (st && tid == 0) {
        st[2] = wall_clock64();
        st[7] = guard;
    }
    // ---- 4. final phase (cc:888-971)
    while (!finish && final_phase) {
        if (++guard > 4096) { if (tid == 0) atomicOr(&status[f], kStatusIterations); break; }
        const NodeBuf& A = cur ? nb1 : nb0;
        const NodeBuf& B = cur ? nb0 : nb1;
        const int prev = size;
        // processing order: vPrev sorted ascending by (size, address), walked from the back.
        // The vPrev members are compacted (block scan) with their order keys (size,
        // creation rank) -- distinct, creation ranks are -- into `best` (free until
        // phase 5), node ids in sb; a member's rank is the number of larger keys among
        // the nv members only, counted over the dense list with independent partial sums.
        for (int j = tid; j < size; j += 256) {
            sa[j] = A.inV[j] ? 1 : 0;
            sc[j] = -1;  // rank of node j in processing order, -1 if not in vPrev
            ccnt[2 * j] = ccnt[2 * j + 1] = 0u;
        }
        __syncthreads();
        const int nv = block_exscan(sa, size, s_tmp);
        if (nv == 0) { finish = true; break; }
        for (int j = tid; j < size; j += 256)
            if (A.inV[j]) {
                best[sa[j]] = ((uint32_t)A.cnt[j] << 16) | (uint32_t)(uint16_t)A.crank[j];
                sb[sa[j]] = j;
            }
        // pad to a multiple of 16 with keys never larger (past NC they land in ccnt, which
        // is zero here)
        if (tid < 15) best[nv + tid] = 0u;
        __syncthreads();
        const unsigned long long t_rank = st && tid == 0 ? wall_clock64() : 0;
        // a member's rank counts the larger keys: two members per thread and pass, the keys
        // read 16 at a time as four broadcast 16-byte LDS reads (latency, not the compares,
        // bounds this loop in a workgroup that has its CU to itself)
        for (int p0 = tid; p0 < nv; p0 += 512) {
            const int p1 = p0 + 256;
            const uint32_t k0 = best[p0], k1 = p1 < nv ? best[p1] : ~0u;
            int r0 = 0, r1 = 0;
            const uint4* b4 = (const uint4*)best;
            for (int i = 0; i < nv; i += 16) {
                uint4 v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) v[u] = b4[(i >> 2) + u];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    r0 += (v[u].x > k0) + (v[u].y > k0) + (v[u].z > k0) + (v[u].w > k0);
                    r1 += (v[u].x > k1) + (v[u].y > k1) + (v[u].z > k1) + (v[u].w > k1);
                }
            }
            sc[sb[p0]] = (int16_t)r0;
            if (p1 < nv) sc[sb[p1]] = (int16_t)r1;
        }
        __syncthreads();
        if (st && tid == 0) st[8] += wall_clock64() - t_rank;
        for (int j = tid; j < size; j += 256)
            if (sc[j] >= 0) sa[sc[j]] = j;  // sa[r] = node processed r-th
        FOR_KEYS({
            const int nd = NN;
            if (A.inV[nd]) {
                const int q = quadrant(key_x(KK), key_y(KK), A.x0[nd], A.y0[nd], A.x1[nd], A.y1[nd]);
                add_q(ccnt, nd, q);
            }
        })
        __syncthreads();
        // sb[r] = ne of the r-th processed node
        for (int r = tid; r < nv; r += 256) {
            const int j = sa[r];
            int ne = 0;
            for (int q = 0; q < 4; q++) ne += get_q(ccnt, j, q) > 0;
            sb[r] = ne;
        }
        // K = first r where prev + sum_{i<=r}(ne_i - 1) >= N (break after it), else nv-1.
        // Every processed node has ne >= 1, so the partial sums never decrease and K is
        // the number of r whose sum stays below N (capped at nv - 1): a block scan of
        // ne - 1 (into sa, free now) and a count instead of a one-thread walk.
        if (tid == 0) s_scal[3] = 0;
        for (int r = tid; r < nv; r += 256) sa[r] = sb[r] - 1;  // sb[r]: this thread's own entry
        __syncthreads();  // block_exscan reads contiguous runs, not the strided entries written here
        block_exscan(sa, nv, s_tmp);
        int below = 0;
        for (int r = tid; r < nv; r += 256) below += prev + sa[r] + sb[r] - 1 < N;
        if (below) atomicAdd(&s_scal[3], below);
        __syncthreads();
        const int Kp = min(s_scal[3], nv - 1);
        const int inclK = sa[Kp] + sb[Kp] - 1;
        const int Cc = inclK + Kp + 1;    // children created
        const int nsize = prev + inclK;   // new size
        if (nsize > NC) { if (tid == 0) atomicOr(&status[f], kStatusNodeOverflow); finish = true; break; }
        // exclusive scan of ne over processing order -> creation ranks / blocks
        const int E_total = block_exscan(sb, Kp + 1, s_tmp);
        (void)E_total;
        // processed flag per node, then position of unprocessed nodes
        for (int j = tid; j < size; j += 256) {
            const int r = sc[j];
            sc[j] = (int16_t)((r >= 0 && r <= Kp) ? r : -1);
        }
        __syncthreads();
        // D_j = number of processed nodes before j (list order)
        for (int j = tid; j < size; j += 256) sa[j] = sc[j] >= 0 ? 1 : 0;
        __syncthreads();
        block_exscan(sa, size, s_tmp);
        for (int j = tid; j < size; j += 256) {
            const int r = sc[j];
            if (r < 0) {
                const int pos = Cc + j - sa[j];
                B.x0[pos] = A.x0[j];
                B.y0[pos] = A.y0[j];
                B.x1[pos] = A.x1[j];
                B.y1[pos] = A.y1[j];
                B.cnt[pos] = A.cnt[j];
                B.crank[pos] = A.crank[j];
                B.inV[pos] = 0;
                sa[j] = pos;
            } else {
                int ne = 0;
                for (int q = 0; q < 4; q++) ne += get_q(ccnt, j, q) > 0;
                const int Er = sb[r];
                const int Bk = Cc - Er - ne;
                int rr = 0;
                for (int q = 0; q < 4; q++) {
                    const int cq = get_q(ccnt, j, q);
                    if (cq > 0) {
                        const int pos = Bk + (ne - 1 - rr);
                        int cx0, cy0, cx1, cy1;
                        child_box(q, A.x0[j], A.y0[j], A.x1[j], A.y1[j], cx0, cy0, cx1, cy1);
                        B.x0[pos] = (int16_t)cx0;
                        B.y0[pos] = (int16_t)cy0;
                        B.x1[pos] = (int16_t)cx1;
                        B.y1[pos] = (int16_t)cy1;
                        B.cnt[pos] = (uint16_t)cq;
                        B.crank[pos] = (int16_t)(Er + rr);
                        B.inV[pos] = cq > 1;
                        cpos[4 * j + q] = (uint16_t)pos;
                        rr++;
                    }
                }
            }
        }
        __syncthreads();
        FOR_KEYS({
            const int nd = NN;
            if (sc[nd] >= 0) {
                const int q = quadrant(key_x(KK), key_y(KK), A.x0[nd], A.y0[nd], A.x1[nd], A.y1[nd]);
                NN = cpos[4 * nd + q];
            } else {
                NN = sa[nd];
            }
        })
        __syncthreads();
        cur ^= 1;
        size = nsize;
        if (size >= N || size == prev) finish = true;
    }

    if (st && tid == 0) st[3] = wall_clock64();
    // ---- 5. best key per node (cc:984-1009)
    for (int j = tid; j < size; j += 256) best[j] = 0u;
    __syncthreads();
    FOR_KEYS({
        const uint32_t v = ((uint32_t)key_resp(KK) << 24) | (0xffffffu - (uint32_t)k);  // k <= kOctMaxKeys
        atomicMax(&best[NN], v);
    })
#undef FOR_KEYS
    __syncthreads();
    const int outn = size < g.ncap ? size : g.ncap;
    uint32_t* out = kept + (size_t)f * kept_pf + g.out_off;
    for (int j = tid; j < outn; j += 256) {
        const unsigned k = 0xffffffu - (best[j] & 0xffffffu);
        out[j] = K[k];
    }
    if (tid == 0) {
        s_scal[7] = outn;
        kept_count[(size_t)f * L + l] = outn;
        if (size > g.ncap) atomicOr(&status[f], kStatusNodeOverflow);
        if (st) {
            st[4] = wall_clock64();
            st[5] = guard;
        }
    }
    };
    if (n <= kOctKeysReg) tail(std::true_type{});
    else tail(std::false_type{});

    // k_describe_tiles' bins: the kept slots of every level tile (k_level_tiles' 64 x 48
    // grid), counted, then listed tile after tile (any order inside a tile: each slot's
    // output position is its own).  The node arrays sa / sb are free now; the host checks
    // that a level's tiles fit in NC entries.
    if (dt_list) {
        const int ntl = g.tiles_x * g.tiles_y;
        int* const tcnt = sa;
        int* const tnum = sb;
        auto tile_of = [&](uint32_t kk) {
            return (int)((key_y(kk) + kMinBorder) / kLtTH) * g.tiles_x + ((key_x(kk) + kMinBorder) >> 6);
        };
        for (int t = tid; t < ntl; t += 256) tcnt[t] = 0;
        __syncthreads();  // also publishes s_scal[7] and the kept slots written above
        const int outn = s_scal[7];
        const uint32_t* out = kept + (size_t)f * kept_pf + g.out_off;
        for (int j = tid; j < outn; j += 256) atomicAdd(&tcnt[tile_of(out[j])], 1);
        __syncthreads();
        for (int t = tid; t < ntl; t += 256) tnum[t] = tcnt[t];
        __syncthreads();
        block_exscan(tcnt, ntl, s_tmp);
        __syncthreads();
        uint32_t* dtt = dt_tile + (size_t)f * tiles_pf + g.tile_first;
        for (int t = tid; t < ntl; t += 256) dtt[t] = ((uint32_t)tcnt[t] << 16) | (uint32_t)tnum[t];
        __syncthreads();
        uint16_t* dl = dt_list + (size_t)f * kept_pf + g.out_off;
        for (int j = tid; j < outn; j += 256) dl[atomicAdd(&tcnt[tile_of(out[j])], 1)] = (uint16_t)j;
    }
}

// ------------------------------------------------------------------ angle + descriptor

// cv::fastAtan2 (OpenCV 3.3.1), degrees; float ops in the reference order.
__device__ float fast_atan2(float y, float x) {
    const float deg = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * deg;
    const float p3 = -0.3258083974640975f * deg;
    const float p5 = 0.1555786518463281f * deg;
    const float p7 = -0.04432655554792128f * deg;
    const float eps = (float)2.2204460492503131e-16;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = __fdiv_rn(ay, ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = __fdiv_rn(ax, ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// Per-level constants of the describe kernels and the frame's kept counts, staged in LDS
// once per workgroup: a slot's level, output base and geometry are then LDS reads, not
// the chain of dependent global loads (one per level passed) of a search over lv[].
struct DescLevel {
    int w, h, pitch;
    uint32_t off;
    int out_off, count;
    float scale, kp_size;
};

__device__ __forceinline__ void stage_desc_levels(DescLevel* s, const LevelGeom* __restrict__ lv,
                                                  const int* __restrict__ kc, int L) {
    const int t = threadIdx.x;
    if (t < L) {
        const LevelGeom& g = lv[t];
        DescLevel d;
        d.w = g.w;
        d.h = g.h;
        d.pitch = g.pitch;
        d.off = (uint32_t)g.off;
        d.out_off = g.out_off;
        d.count = kc[t];
        d.scale = g.scale;
        d.kp_size = g.kp_size;
        s[t] = d;
    }
    __syncthreads();
}

// Level l of kept slot `slot` (out_off is non-decreasing), the output index of the level's
// first keypoint (base) and the frame's keypoint count (total): independent LDS reads.
__device__ __forceinline__ void desc_level_of(const DescLevel* s, int L, int slot, int& l, int& base, int& total) {
    l = 0;
    base = 0;
    total = 0;
    for (int l2 = 0; l2 < L; l2++) {
        const int c = s[l2].count;
        total += c;
        if (l2 + 1 < L && slot >= s[l2 + 1].out_off) {
            base += c;
            l = l2 + 1;
        }
    }
}

// k_describe's staging form by keypoint slots per frame.  Direct-to-LDS staging (more
// describe waves per SIMD) is the faster kernel, alone and in the pipelined configs[1]
// step (222.1-223.8k -> 226.4-227.7k frames/s), but at 5000 features, where the matcher
// beside the extraction sets the step, the extra waves cost the matcher more than they
// save (configs[4] 100.6-100.9k -> 94.1-95.1k; capping them by LDS gives both back):
// register staging above this many slots.
#ifndef ORBX_DESC_GLDS_MAX
// Since round 5 every frame size takes the LDS-DMA form: with lane 1 of a deep pyramid
// (configs[4]) starting after lane 0's FAST cells instead of its octree, the DMA describe
// (0.52-0.62 ms per launch beside the rest, against 1.0 ms) no longer slows the other
// lane's blur: 110.5-111.4k frames/s against 111.0-111.1k for register staging (r05c)
#define ORBX_DESC_GLDS_MAX 1000000
#endif
constexpr int kDescGldsMaxSlots = ORBX_DESC_GLDS_MAX;
#ifndef ORBX_DESC_DMA
// the LDS-DMA form below kDescGldsMaxSlots: 1 = 16-byte pieces into 48-byte rows (five
// workgroups a CU), 2 = 4-byte pieces into 40-byte rows (24.7 KB, six a CU: configs[1]
// pipelined 222.3-224.0k -> 224.5-225.0k frames/s over three interleaved pairs, alone
// 0.209 -> 0.218 ms; KITTI unchanged)
#define ORBX_DESC_DMA 2
#endif

// Four kept keypoint slots per wave (one per 16-lane quarter): IC_Angle on the level
// (cc:59-106), rBRIEF on the blurred level (cc:118-172), coordinate scaling
// (cc:1613-1622), output in the reference's level-major order.  Everything evaluated
// once per wave (fastAtan2, the double-precision sincos, the rounding constants) is
// shared by four keypoints.  (Round 3: two per wave before, one per 32-lane half; four
// take slightly longer alone -- configs[4] 0.654 -> 0.675 ms per launch -- but half the
// waves leave the CUs to the other lane and the matcher: pipelined configs[4] 95.4-95.7k
// -> 100.9-101.3k frames/s, configs[1] 215-218k -> 219.5k.)
//   IC_Angle by rows: a lane reads rows v1 = ql - 15 and v2 = ql + 1 of the level (quarter
//   lane 15 has no second row), 36 bytes from (x-15) & ~3 each, and two v_dot4_u32_u8 per
//   dword against the circular mask and the (u + 15)-weighted mask give sum(I) and
//   sum((u+15) I) over the row: m10 += sum((u+15) I) - 15 sum(I), m01 += v sum(I).
//   The steered-BRIEF patch of the blurred level, rows y-18..y+18 (|rotated pattern
//   point| <= 13*sqrt(2) < 18.5), 44 bytes from (x-18) & ~3, is staged in LDS as 111
//   16-byte chunks (48-byte rows); all global loads are issued together, one round of
//   latency.  STAGE 1 / 2: the patch goes straight to LDS (global_load_lds_dwordx4 /
//   _dword, no VGPR destinations: 76-78 instead of 102 VGPRs, five / six waves per SIMD
//   instead of four); STAGE 0: through registers, seven chunks per lane.  Keypoints lie in [19, w-20] x [19, h-20] of their level, so
//   every row exists; a row's last dword may reach 6 bytes past the level width (inside
//   the pitch, or the buffers' slack for the very last row).
//   A lane samples 16 of the 256 pairs (ql, 16 + ql, ..., 240 + ql); each pair step's
//   ballot carries 16 descriptor bits per keypoint.
template <int STAGE>  // 0: registers, 1: 16-byte LDS-DMA, 2: 4-byte LDS-DMA into 40-byte rows
__global__ __launch_bounds__(256) void k_describe(const uint8_t* __restrict__ pyr,
                                                   const uint8_t* __restrict__ blur, long long fb,
                                                   const LevelGeom* __restrict__ lv, int L,
                                                   const uint32_t* __restrict__ kept, int kept_pf,
                                                   const int* __restrict__ kept_count,
                                                   orbx_keypoint* __restrict__ kps, uint8_t* __restrict__ desc,
                                                   int cap, int* __restrict__ n_out, int nframes,
                                                   const uint8_t* __restrict__ l0, long long l0_fp, int l0_pitch,
                                                   const int* __restrict__ status, int* __restrict__ status_out) {
    // BRIEF patches: 37 rows of 48 bytes (16-byte chunks), or of 40 bytes -- the 37
    // columns x-18..x+18 from (x-18) & ~3 -- for the 4-byte DMA (six workgroups a CU)
    constexpr int kPP = STAGE == 2 ? 40 : 48;
    __shared__ __align__(16) uint32_t s_bpatch[16][37 * kPP / 4];
    __shared__ DescLevel s_lv[kMaxLevels];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int qt = lane >> 4, ql = lane & 15;
    int f, sb;
    xcd_frame_block((kept_pf + 15) / 16, nframes, f, sb);
    const int slot0 = sb * 16 + wave * 4;
    const int slot = slot0 + qt;
    const uint32_t key_raw = kept[(size_t)f * kept_pf + min(slot, kept_pf - 1)];
    stage_desc_levels(s_lv, lv, kept_count + (size_t)f * L, L);
    if (slot0 >= kept_pf) return;  // whole wave; no barriers below
    int l, base, total;
    desc_level_of(s_lv, L, slot, l, base, total);
    if (slot0 == 0 && lane == 0) {
        n_out[f] = total;
        if (status_out) status_out[f] = status[f];  // k_octree's word (earlier on this stream)
    }
    const DescLevel& g = s_lv[l];
    const int i = slot - g.out_off;
    const int o = base + i;
    const bool valid = slot < kept_pf && i < g.count && o < cap;
    if (__ballot(valid) == 0) return;  // all four quarters empty
    const uint32_t key = valid ? key_raw : 0u;
    // an empty quarter samples the middle of its level (>= 23 px from every edge) and is masked
    const int x = valid ? key_x(key) + kMinBorder : g.w / 2;
    const int y = valid ? key_y(key) + kMinBorder : g.h / 2;
    const int resp = key_resp(key);
    const int pitch = g.pitch;
    float lv_scale = g.scale, lv_size = g.kp_size;
    asm volatile("" : "+v"(lv_scale), "+v"(lv_size));
    const int kp = wave * 4 + qt;
    uint8_t* const bp = (uint8_t*)s_bpatch[kp];
    const int xs = (x - 15) & ~3, xb = (x - 18) & ~3;
    int m10, m01;
    {
        const uint8_t* bframe = blur + (size_t)f * fb;
        // the IC rows' level: level 0 from the input frame when it is read in place
        const bool in0 = l == 0 && l0 != nullptr;
        const uint8_t* plevel = in0 ? l0 + (size_t)f * l0_fp : pyr + (size_t)f * fb + g.off;
        const int rpitch = in0 ? l0_pitch : pitch;
        // rows v1 = ql - 15 (-15..0) and v2 = ql + 1 (1..15; quarter lane 15 has none)
        const int v1 = ql - 15, v2 = min(ql + 1, 15);
        const int d0 = (x - 15) & 3;
        const uint8_t* prow1 = plevel + (uint32_t)((y + v1) * rpitch + xs);
        const uint8_t* prow2 = plevel + (uint32_t)((y + v2) * rpitch + xs);
        const uint4 p0 = *(const uint4*)prow1, p1 = *(const uint4*)(prow1 + 16);
        const uint32_t p2 = *(const uint32_t*)(prow1 + 32);
        const uint4 r0 = *(const uint4*)prow2, r1 = *(const uint4*)(prow2 + 16);
        const uint32_t r2 = *(const uint32_t*)(prow2 + 32);
        const uint8_t* bpatch = bframe + (uint32_t)(g.off + (long long)(y - 18) * pitch + xb);
        if constexpr (STAGE == 1) {
        // the four BRIEF patches go straight to LDS (global_load_lds_dwordx4: no VGPR
        // destinations, so more waves fit a SIMD): patch by patch, the whole wave loads
        // its 111 chunks (lane L chunks L and 64 + L), from the patch base of quarter q
        // read off lane 16 q; an LDS-DMA piece lands at base + 16 x lane
        {
            const uint64_t mybase = (uint64_t)(uintptr_t)bpatch;
            uint8_t* const wbp = (uint8_t*)s_bpatch[wave * 4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)mybase, 16 * q);
                const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(mybase >> 32), 16 * q);
                const int sp = __builtin_amdgcn_readlane(pitch, 16 * q);
                const uint8_t* qb = (const uint8_t*)(uintptr_t)(((uint64_t)hi << 32) | lo);
#pragma unroll
                for (int jj = 0; jj < 2; jj++) {
                    const int c = 64 * jj + lane;
                    if (c < 111) {
                        const int row = (c * 171) >> 9;
                        __builtin_amdgcn_global_load_lds((const void*)(qb + (uint32_t)(row * sp + 16 * (c - 3 * row))),
                                                         (__attribute__((address_space(3))) void*)(wbp + q * (int)sizeof(s_bpatch[0]) + 1024 * jj),
                                                         16, 0, 0);
                    }
                }
            }
        }
        }
        if constexpr (STAGE == 2) {
            // 4-byte pieces: patch q's 370 dwords (37 rows x 10), lane L dword L + 64 j
            const uint64_t mybase = (uint64_t)(uintptr_t)bpatch;
            uint8_t* const wbp = (uint8_t*)s_bpatch[wave * 4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)mybase, 16 * q);
                const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(mybase >> 32), 16 * q);
                const int sp = __builtin_amdgcn_readlane(pitch, 16 * q);
                const uint8_t* qb = (const uint8_t*)(uintptr_t)(((uint64_t)hi << 32) | lo);
#pragma unroll
                for (int jj = 0; jj < 6; jj++) {
                    const int c = 64 * jj + lane;
                    if (c < 370) {
                        const int row = (c * 205) >> 11;  // c / 10 for c < 370
                        __builtin_amdgcn_global_load_lds((const void*)(qb + (uint32_t)(row * sp + 4 * (c - 10 * row))),
                                                         (__attribute__((address_space(3))) void*)(wbp + q * (int)sizeof(s_bpatch[0]) + 256 * jj),
                                                         4, 0, 0);
                    }
                }
            }
        }
        uint4 bch[7];
        if constexpr (STAGE == 0) {
#pragma unroll
            for (int j = 0; j < 7; j++) {
                const int c = min(ql + 16 * j, 110), row = (c * 171) >> 9;
                bch[j] = *(const uint4*)(bpatch + (uint32_t)(row * pitch + 16 * (c - 3 * row)));
            }
        }
        auto row_sums = [&](const uint4& a0, const uint4& a1, uint32_t a2, int av, uint32_t& cs, uint32_t& ws) {
            const uint4* cm = (const uint4*)c_icm[d0][av];
            const uint4* cw = (const uint4*)c_icw[d0][av];
            const uint4 m0 = cm[0], m1 = cm[1], m2 = cm[2], w0 = cw[0], w1 = cw[1], w2 = cw[2];
            cs = 0;
            ws = 0;
            cs = __builtin_amdgcn_udot4(a0.x, m0.x, cs, false); ws = __builtin_amdgcn_udot4(a0.x, w0.x, ws, false);
            cs = __builtin_amdgcn_udot4(a0.y, m0.y, cs, false); ws = __builtin_amdgcn_udot4(a0.y, w0.y, ws, false);
            cs = __builtin_amdgcn_udot4(a0.z, m0.z, cs, false); ws = __builtin_amdgcn_udot4(a0.z, w0.z, ws, false);
            cs = __builtin_amdgcn_udot4(a0.w, m0.w, cs, false); ws = __builtin_amdgcn_udot4(a0.w, w0.w, ws, false);
            cs = __builtin_amdgcn_udot4(a1.x, m1.x, cs, false); ws = __builtin_amdgcn_udot4(a1.x, w1.x, ws, false);
            cs = __builtin_amdgcn_udot4(a1.y, m1.y, cs, false); ws = __builtin_amdgcn_udot4(a1.y, w1.y, ws, false);
            cs = __builtin_amdgcn_udot4(a1.z, m1.z, cs, false); ws = __builtin_amdgcn_udot4(a1.z, w1.z, ws, false);
            cs = __builtin_amdgcn_udot4(a1.w, m1.w, cs, false); ws = __builtin_amdgcn_udot4(a1.w, w1.w, ws, false);
            cs = __builtin_amdgcn_udot4(a2, m2.x, cs, false); ws = __builtin_amdgcn_udot4(a2, w2.x, ws, false);
        };
        uint32_t cs1, ws1, cs2, ws2;
        row_sums(p0, p1, p2, -v1, cs1, ws1);
        row_sums(r0, r1, r2, v2, cs2, ws2);
        const bool row2_ok = ql < 15;
        m10 = ((int)ws1 - 15 * (int)cs1) + (row2_ok ? (int)ws2 - 15 * (int)cs2 : 0);
        m01 = v1 * (int)cs1 + (row2_ok ? v2 * (int)cs2 : 0);
        if constexpr (STAGE != 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA pieces have landed
        } else {
#pragma unroll
            for (int j = 0; j < 7; j++)
                if (ql + 16 * j < 111) ((uint4*)bp)[ql + 16 * j] = bch[j];  // chunk c at byte 16 c
        }
    }
    wave_lds_fence();
#pragma unroll
    for (int o2 = 8; o2 > 0; o2 >>= 1) {  // within the 16-lane quarter
        m10 += __shfl_xor(m10, o2);
        m01 += __shfl_xor(m01, o2);
    }
    const float angle = fast_atan2((float)m01, (float)m10);

    const float factorPI = (float)(3.14159265358979323846 / 180.f);
    const float rad = angle * factorPI;
    double cd, sd;
    sincos_0_2pi((double)rad, cd, sd);  // == (float)cos/sin((double)rad) (orbx_sincos.h)
    const float a = (float)cd, b = (float)sd;
    // cvRound(v) for |v| < 2^22 is the low bits of v + 1.5 * 2^23 (round to nearest
    // even, like rint): 0x4B400000 + cvRound(v).  The row offset is one v_mul_u32_u24,
    // which reads only the low 24 bits (0x400000 + cvRound(y)); the constants come off
    // the patch centre once.
    const uint32_t center = (uint32_t)(18 * kPP + 18 + (x - 18 - xb)) - (0x400000u * (uint32_t)kPP + 0x4B400000u);
    const float kRound = 12582912.0f;  // 1.5 * 2^23
    // the offsets fused as g++ -O3 -march=native builds the reference (hazard H4: GCC
    // contracts C++ and fuses the first product, fma(x, b, y*a), fma(x, a, -(y*b)))
    auto sample = [&](float px, float py) -> int {
        const uint32_t ry = __float_as_uint(fmaf(px, b, py * a) + kRound);
        const uint32_t rx = __float_as_uint(fmaf(px, a, -(py * b)) + kRound);
        return bp[center + __umul24(ry, (uint32_t)kPP) + rx];
    };
    auto pair_test = [&](int q) -> bool {
        const float x0 = (float)(int8_t)(q & 0xff), y0 = (float)(int8_t)((q >> 8) & 0xff);
        const float x1 = (float)(int8_t)((q >> 16) & 0xff), y1 = (float)(int8_t)(q >> 24);
        return sample(x0, y0) < sample(x1, y1);
    };
    int pat[16];
#pragma unroll
    for (int v = 0; v < 4; v++) {
        const int4 p4 = ((const int4*)c_pattern[ql])[v];
        pat[4 * v] = p4.x;
        pat[4 * v + 1] = p4.y;
        pat[4 * v + 2] = p4.z;
        pat[4 * v + 3] = p4.w;
    }
    // descriptor word w (pairs 32 w .. 32 w + 31) = this quarter's 16 bits of the ballots
    // of pair steps 2 w and 2 w + 1; lane ql < 2 stores words 4 ql .. 4 ql + 3
    const int qsh = 16 * (qt & 1);
    uint32_t words[8];
#pragma unroll
    for (int w = 0; w < 8; w++) {
        const unsigned long long ba = __ballot(pair_test(pat[2 * w]));
        const unsigned long long bb = __ballot(pair_test(pat[2 * w + 1]));
        const uint32_t la = (qt & 2) ? (uint32_t)(ba >> 32) : (uint32_t)ba;
        const uint32_t lb = (qt & 2) ? (uint32_t)(bb >> 32) : (uint32_t)bb;
        words[w] = ((la >> qsh) & 0xffffu) | ((lb >> qsh) << 16);
    }
    if (valid && ql < 2) {
        uint4* d = (uint4*)(desc + ((size_t)f * cap + o) * 32);
        d[ql] = ql == 0 ? make_uint4(words[0], words[1], words[2], words[3])
                        : make_uint4(words[4], words[5], words[6], words[7]);
    }
    if (valid && ql == 0) {
        float fx = (float)x, fy = (float)y;
        if (l != 0) {
            fx = fx * lv_scale;
            fy = fy * lv_scale;
        }
        orbx_keypoint kpo;
        kpo.x = fx;
        kpo.y = fy;
        kpo.size = lv_size;
        kpo.angle = angle;
        kpo.response = (float)resp;
        kpo.octave = l;
        kpo.class_id = -1;
        kps[(size_t)f * cap + o] = kpo;
    }
}

// Tile-major describe (dense frames: configs[4]'s 5000 keypoints, ~16 per level tile).
// One workgroup per level tile of k_level_tiles' 64 x 48 grid: the tile plus an 18-px
// halo of the level (rows Y0-18 .. Y0+65, 128 columns from (X0-18) & ~15) is staged in
// LDS once, raw and blurred, in 16-byte row loads, and every kept keypoint the octree
// binned into the tile is described from there: IC_Angle's rows (cc:59-106) and the
// rBRIEF samples (cc:118-172) become LDS reads, instead of each keypoint staging its own
// 37 x 37 blurred patch and 31 raw rows (k_describe: ~2.6 KB per keypoint, 6x a dense
// frame's two images).  Four keypoints per wave as in k_describe, 16 per round.
constexpr int kDtP = 128;               // staged row pitch (bytes)
constexpr int kDtRows = kLtTH + 36;     // tile rows + 18-px halo above and below
__global__ __launch_bounds__(256) void k_describe_tiles(const uint8_t* __restrict__ pyr,
                                                         const uint8_t* __restrict__ blur, long long fb,
                                                         const LevelGeom* __restrict__ lv, int L,
                                                         const uint32_t* __restrict__ kept, int kept_pf,
                                                         const int* __restrict__ kept_count,
                                                         const uint16_t* __restrict__ dt_list,
                                                         const uint32_t* __restrict__ dt_tile, int tiles_pf,
                                                         orbx_keypoint* __restrict__ kps, uint8_t* __restrict__ desc,
                                                         int cap, int* __restrict__ n_out, int nframes,
                                                         const int* __restrict__ status, int* __restrict__ status_out) {
    __shared__ __align__(16) uint8_t s_raw[kDtRows][kDtP];
    __shared__ __align__(16) uint8_t s_blr[kDtRows][kDtP];
    int f, tile;
    xcd_frame_block(tiles_pf, nframes, f, tile);
    const int tid = threadIdx.x;
    const int* kc = kept_count + (size_t)f * L;
    if (tile == 0 && tid == 0) {
        int tot = 0;
        for (int l2 = 0; l2 < L; l2++) tot += kc[l2];
        n_out[f] = tot;
        if (status_out) status_out[f] = status[f];
    }
    const uint32_t td = dt_tile[(size_t)f * tiles_pf + tile];
    const int cnt = (int)(td & 0xffffu), start = (int)(td >> 16);
    if (cnt == 0) return;  // whole workgroup, before any barrier
    int l = 0;
    while (l + 1 < L && tile >= lv[l + 1].tile_first) l++;
    const LevelGeom& g = lv[l];
    int base = 0;  // output index of the level's first keypoint
    for (int l2 = 0; l2 < l; l2++) base += kc[l2];
    const int t = tile - g.tile_first;
    const int ty = t / g.tiles_x;
    const int X0 = (t - ty * g.tiles_x) * kLtTW, Y0 = ty * kLtTH;
    const int Xs = max(0, (X0 - 18) & ~15), Ys = max(0, Y0 - 18);
    const int nrows = min(g.h, Y0 + kLtTH + 18) - Ys;
    const int nch = (min(g.w, X0 + kLtTW + 18) - Xs + 15) >> 4;  // 16-byte chunks per row (<= 8)
    {
        // all loads of a thread issued before its LDS stores; chunks past the level's
        // right edge are not loaded (nothing samples them)
        constexpr int kPer = (kDtRows * (kDtP / 16) + 255) / 256;
        const uint8_t* pr = pyr + (size_t)f * fb + g.off + (size_t)Ys * g.pitch + Xs;
        const uint8_t* br = blur + (size_t)f * fb + g.off + (size_t)Ys * g.pitch + Xs;
        // (a thread past the region loads and stores the region's last chunk again)
        uint4 a[kPer], b[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int i = tid + 256 * k;
            const int r = min(i >> 3, nrows - 1), c = min(i & 7, nch - 1);
            const uint32_t o = (uint32_t)(r * g.pitch + 16 * c);
            a[k] = *(const uint4*)(pr + o);
            b[k] = *(const uint4*)(br + o);
        }
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const int i = tid + 256 * k;
            const int r = min(i >> 3, nrows - 1), c = min(i & 7, nch - 1);
            *(uint4*)&s_raw[r][16 * c] = a[k];
            *(uint4*)&s_blr[r][16 * c] = b[k];
        }
    }
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int qt = lane >> 4, ql = lane & 15;
    const uint32_t* kl = kept + (size_t)f * kept_pf + g.out_off;
    const uint16_t* dl = dt_list + (size_t)f * kept_pf + g.out_off + start;
    float lv_scale = g.scale, lv_size = g.kp_size;
    for (int s0 = wave * 4; s0 < cnt; s0 += 16) {  // wave-uniform; no barriers below
        const int s = s0 + qt;
        const bool in = s < cnt;
        const int j = in ? dl[s] : 0;
        const int o = base + j;
        const bool valid = in && o < cap;
        const uint32_t key = kl[j];
        // an empty quarter samples the tile's first keypoint and is masked
        const int x = key_x(valid ? key : kl[dl[0]]) + kMinBorder;
        const int y = key_y(valid ? key : kl[dl[0]]) + kMinBorder;
        const int resp = key_resp(key);
        // IC_Angle: rows v1 = ql - 15 and v2 = ql + 1 (quarter lane 15 has none), 36 bytes
        // from (x - 15) & ~3 as nine dword LDS reads each
        const int v1 = ql - 15, v2 = min(ql + 1, 15);
        const int d0 = (x - 15) & 3;
        const int cs0 = ((x - 15) & ~3) - Xs;
        auto row_sums = [&](int rr, int av, uint32_t& cs, uint32_t& ws) {
            const uint32_t* rp = (const uint32_t*)&s_raw[rr][cs0];
            const uint4* cm4 = (const uint4*)c_icm[d0][av];
            const uint4* cw4 = (const uint4*)c_icw[d0][av];
            const uint4 m0 = cm4[0], m1 = cm4[1], m2 = cm4[2], w0 = cw4[0], w1 = cw4[1], w2 = cw4[2];
            const uint32_t cm[9] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w, m2.x};
            const uint32_t cw[9] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x};
            cs = 0;
            ws = 0;
#pragma unroll
            for (int k = 0; k < 9; k++) {
                const uint32_t d = rp[k];
                cs = __builtin_amdgcn_udot4(d, cm[k], cs, false);
                ws = __builtin_amdgcn_udot4(d, cw[k], ws, false);
            }
        };
        uint32_t cs1, ws1, cs2, ws2;
        row_sums(y + v1 - Ys, -v1, cs1, ws1);
        row_sums(y + v2 - Ys, v2, cs2, ws2);
        const bool row2_ok = ql < 15;
        int m10 = ((int)ws1 - 15 * (int)cs1) + (row2_ok ? (int)ws2 - 15 * (int)cs2 : 0);
        int m01 = v1 * (int)cs1 + (row2_ok ? v2 * (int)cs2 : 0);
#pragma unroll
        for (int o2 = 8; o2 > 0; o2 >>= 1) {  // within the 16-lane quarter
            m10 += __shfl_xor(m10, o2);
            m01 += __shfl_xor(m01, o2);
        }
        const float angle = fast_atan2((float)m01, (float)m10);
        const float factorPI = (float)(3.14159265358979323846 / 180.f);
        const float rad = angle * factorPI;
        double cd, sd;
        sincos_0_2pi((double)rad, cd, sd);  // == (float)cos/sin((double)rad) (orbx_sincos.h)
        const float ca = (float)cd, sb = (float)sd;
        // cvRound by the 1.5 * 2^23 bias, as in k_describe, over the staged blurred tile
        const uint8_t* bp = &s_blr[0][0];
        const uint32_t center = (uint32_t)((y - Ys) * kDtP + (x - Xs)) - (0x400000u * (uint32_t)kDtP + 0x4B400000u);
        const float kRound = 12582912.0f;
        auto sample = [&](float px, float py) -> int {  // fused like the reference's build (H4)
            const uint32_t ry = __float_as_uint(fmaf(px, sb, py * ca) + kRound);
            const uint32_t rx = __float_as_uint(fmaf(px, ca, -(py * sb)) + kRound);
            return bp[center + __umul24(ry, (uint32_t)kDtP) + rx];
        };
        auto pair_test = [&](int q) -> bool {
            const float x0 = (float)(int8_t)(q & 0xff), y0 = (float)(int8_t)((q >> 8) & 0xff);
            const float x1 = (float)(int8_t)((q >> 16) & 0xff), y1 = (float)(int8_t)(q >> 24);
            return sample(x0, y0) < sample(x1, y1);
        };
        int pat[16];
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int4 p4 = ((const int4*)c_pattern[ql])[v];
            pat[4 * v] = p4.x;
            pat[4 * v + 1] = p4.y;
            pat[4 * v + 2] = p4.z;
            pat[4 * v + 3] = p4.w;
        }
        const int qsh = 16 * (qt & 1);
        uint32_t words[8];
#pragma unroll
        for (int w = 0; w < 8; w++) {
            const unsigned long long ba = __ballot(pair_test(pat[2 * w]));
            const unsigned long long bb = __ballot(pair_test(pat[2 * w + 1]));
            const uint32_t la = (qt & 2) ? (uint32_t)(ba >> 32) : (uint32_t)ba;
            const uint32_t lb = (qt & 2) ? (uint32_t)(bb >> 32) : (uint32_t)bb;
            words[w] = ((la >> qsh) & 0xffffu) | ((lb >> qsh) << 16);
        }
        if (valid && ql < 2) {
            uint4* d = (uint4*)(desc + ((size_t)f * cap + o) * 32);
            d[ql] = ql == 0 ? make_uint4(words[0], words[1], words[2], words[3])
                            : make_uint4(words[4], words[5], words[6], words[7]);
        }
        if (valid && ql == 0) {
            float fx = (float)x, fy = (float)y;
            if (l != 0) {
                fx = fx * lv_scale;
                fy = fy * lv_scale;
            }
            orbx_keypoint kpo;
            kpo.x = fx;
            kpo.y = fy;
            kpo.size = lv_size;
            kpo.angle = angle;
            kpo.response = (float)resp;
            kpo.octave = l;
            kpo.class_id = -1;
            kps[(size_t)f * cap + o] = kpo;
        }
    }
}

// ------------------------------------------------------------------ host launch

hipError_t launch_extract(const Plan& plan, const DeviceBuffers& db, int batch, const uint8_t* d_imgs,
                          size_t frame_pitch, size_t stride, void* kps, uint8_t* desc, int cap,
                          int* n_per_frame, hipStream_t stream, hipEvent_t* ev, hipEvent_t stage_ev,
                          int stage_after, bool l0_in_place, int* status_out) {
    // level 0 read in place by k_level_tiles / k_describe (their 16-byte row loads need
    // 16-byte aligned frames and 64-byte aligned rows), not copied into the pyramid
    const uint8_t* l0 = l0_in_place ? d_imgs : nullptr;
    const long long l0_fp = (long long)frame_pitch;
    const int l0_pitch = (int)stride;
    const int L = plan.L;
    const long long fb = plan.pyr_frame_bytes;
    const int ncells = (int)plan.cells.size();
    // switch dup_stage = k (measurement): launch stage k (1 pyramid .. 5 describe) twice --
    // every stage is idempotent -- so a pipelined run prices that stage's marginal cost
    const int dup = tuning(Tune::DupStage, 0);
    if (ev && ev[0]) (void)hipEventRecord(ev[0], stream);
    for (int rep = 0; rep < (dup == 1 ? 2 : 1); rep++) {
        // one launch per pyramid segment (orbx_geometry.h): the first reads the input
        // frames, a later one its input level from the pyramid the previous one wrote
        auto kern = plan.pz_win ? k_pyramid<true> : k_pyramid<false>;
        size_t lds_max = 0;
        for (int s = 0; s < plan.pz_nseg; s++)
            lds_max = std::max(lds_max, (size_t)plan.pz[s].lds_a + plan.pz[s].lds_b);
        if (lds_max > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max);
            if (e != hipSuccess) return e;
        }
        for (int s = 0; s < plan.pz_nseg; s++) {
            const PzSeg& sg = plan.pz[s];
            const LevelGeom& g0 = plan.lv[sg.l0];
            const uint8_t* in = s == 0 ? d_imgs : db.pyr + g0.off;
            const size_t fp = s == 0 ? frame_pitch : (size_t)fb, st = s == 0 ? stride : (size_t)g0.pitch;
            const int vec4 = ((uintptr_t)in % 4 == 0) && (st % 4 == 0) && (fp % 4 == 0);
            hipLaunchKernelGGL(kern, dim3(sg.tiles * batch), dim3(256), (size_t)sg.lds_a + sg.lds_b, stream, in, fp, st,
                               vec4, db.pyr, fb, db.lv + sg.l0, sg.nl, db.rtab, sg.off, sg.tiles, batch, sg.lds_a,
                               db.status, (s == 0 && l0) ? 0 : 1);
        }
    }
    if (ev && ev[1]) (void)hipEventRecord(ev[1], stream);
    if (stage_ev && stage_after == 1) (void)hipEventRecord(stage_ev, stream);
    for (int rep = 0; rep < (dup == 2 ? 2 : 1); rep++) {
        dim3 grid(plan.tiles_total * batch);
        int tq = plan.prm.ini_th < plan.prm.min_th ? plan.prm.ini_th : plan.prm.min_th;
        tq = tq < 0 ? 0 : (tq > 255 ? 255 : tq);
        hipLaunchKernelGGL(k_level_tiles, grid, dim3(256), 0, stream, db.pyr, db.blur, db.score, fb, db.lv, L,
                           plan.tiles_total, batch, tq, l0, l0_fp, l0_pitch);
    }
    if (ev && ev[2]) (void)hipEventRecord(ev[2], stream);
    if (stage_ev && stage_after == 2) (void)hipEventRecord(stage_ev, stream);
    for (int rep = 0; rep < (dup == 3 ? 2 : 1); rep++) {
        dim3 grid(((ncells + 3) / 4) * batch);
        if (plan.fc_wc + 2 > kFcStride) return hipErrorInvalidValue;  // a window wider than the staged pitch
        const size_t fc_lds = 4 * (size_t)((((plan.fc_wr + 2) * kFcStride + 2 * plan.fc_wr * plan.fc_wc) + 15) & ~15);
        hipLaunchKernelGGL(k_fast_cells, grid, dim3(256), fc_lds, stream, db.score, fb, db.cells, ncells,
                           plan.prm.ini_th, plan.prm.min_th, db.slots, plan.slots_per_frame, db.cell_count, batch,
                           plan.fc_wr, plan.fc_wc);
    }
    if (ev && ev[3]) (void)hipEventRecord(ev[3], stream);
    if (stage_ev && stage_after == 3) (void)hipEventRecord(stage_ev, stream);
    for (int rep = 0; rep < (dup == 4 ? 2 : 1); rep++) {
        // A launch's dynamic LDS is sized for its largest level.  For a batch whose level-0
        // node table is large enough to limit the workgroups per CU (over 32 KB: fewer than
        // the 5 its registers allow), the levels whose node capacity is at most 3/8 of level
        // 0's go in a second launch sized for them (configs[4]: levels 6-11 at 15 KB instead
        // of 46 KB), so those workgroups hold less LDS beside the other kernels on their CU:
        // configs[4] 107.4-108.9k -> 114.8-115.2k frames/s.  Splitting earlier leaves the
        // first launch too few workgroups to cover its tail (after level 1: 102.6k; after 3:
        // 111.4-112.0k; after 4: 113.2-114.5k; r05t-v).  Without a large table the second
        // launch only serialises the stage (configs[1] 226.5k -> 219.3k, KITTI -2.6 %; r05s).
        int split = L;
        const bool big = (size_t)((plan.max_ncap + 63) & ~63) * kOctNodeBytes > 32 * 1024;
        if (batch >= 16 && big && !plan.desc_tiles && kOctSplitLevels)
            for (int l = 1; l < L; l++)
                if (plan.lv[l].ncap * ORBX_OCT_SPLIT_DEN <= plan.lv[0].ncap * ORBX_OCT_SPLIT_NUM) {
                    split = l;
                    break;
                }
        for (int part = 0; part < 2; part++) {
            const int la = part ? split : 0, lb = part ? L : split;
            if (la >= lb) continue;
            int mx = 0;
            for (int l = la; l < lb; l++) mx = plan.lv[l].ncap > mx ? plan.lv[l].ncap : mx;
            // the tile-major describe's bins need every level's tiles within NC (one launch)
            const int NC = plan.desc_tiles ? (plan.max_ncap + 63) & ~63 : (mx + 63) & ~63;
            const size_t lds = (size_t)NC * kOctNodeBytes;
            // int16 node ids / ranks, and one workgroup's LDS (beside its static arrays)
            if (NC > 32767 || lds > 152 * 1024) return hipErrorInvalidValue;
            if (lds > 64 * 1024) {
                const hipError_t e =
                    hipFuncSetAttribute((const void*)k_octree, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
                if (e != hipSuccess) return e;
            }
            dim3 grid((lb - la) * batch);
            hipLaunchKernelGGL(k_octree, grid, dim3(256), lds, stream, db.lv, L, db.slots, plan.slots_per_frame,
                               db.cells, db.cell_count, ncells, db.keys, db.key_node, plan.keys_per_frame,
                               db.kept, plan.kept_per_frame, db.kept_count, db.status, NC, batch, db.oct_stamps,
                               plan.desc_tiles ? db.dt_list : nullptr, db.dt_tile, plan.tiles_total, la);
        }
    }
    if (ev && ev[4]) (void)hipEventRecord(ev[4], stream);
    if (stage_ev && stage_after == 4) (void)hipEventRecord(stage_ev, stream);
    for (int rep = 0; rep < (dup == 5 ? 2 : 1); rep++) {
        if (plan.desc_tiles) {
            hipLaunchKernelGGL(k_describe_tiles, dim3(plan.tiles_total * batch), dim3(256), 0, stream, db.pyr,
                               db.blur, fb, db.lv, L, db.kept, plan.kept_per_frame, db.kept_count, db.dt_list,
                               db.dt_tile, plan.tiles_total, (orbx_keypoint*)kps, desc, cap, n_per_frame, batch,
                               db.status, status_out);
        } else {
            dim3 grid(((plan.kept_per_frame + 15) / 16) * batch);
            auto kern = plan.kept_per_frame <= kDescGldsMaxSlots ? k_describe<ORBX_DESC_DMA> : k_describe<0>;
            hipLaunchKernelGGL(kern, grid, dim3(256), 0, stream, db.pyr, db.blur, fb, db.lv, L, db.kept,
                               plan.kept_per_frame, db.kept_count, (orbx_keypoint*)kps, desc, cap, n_per_frame, batch,
                               l0, l0_fp, l0_pitch, db.status, status_out);
        }
    }
    if (ev && ev[5]) (void)hipEventRecord(ev[5], stream);
    return hipGetLastError();
}

}  // namespace orbx
