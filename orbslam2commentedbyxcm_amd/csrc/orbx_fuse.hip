// orbx_fuse.hip -- the remaining Hamming consumers off the per-frame path (SURVEY.md
// §8(f) rank 4):
//   ORBmatcher::Fuse(KeyFrame*, vpMapPoints, th)           ORBmatcher.cc:1067-1221
//   ORBmatcher::Fuse(KeyFrame*, Scw, vpPoints, th, ...)    ORBmatcher.cc:1226-1352
//   ORBmatcher::SearchBySim3                               ORBmatcher.cc:1361-1602
//   MapPoint::ComputeDistinctiveDescriptors                MapPoint.cc:295-360
//
// k_window_best: the searches above take, per projected MapPoint, the first keypoint
// of the keyframe's grid window with the smallest distance, with no claims between
// MapPoints -- so every query is independent.  One 16-lane DPP row per query, four
// per wave; the lanes split the window's column runs of the CSR grid (a column's
// cells are contiguous), keys (dist << 23 | iteration rank) make the DPP row minimum
// the reference's first-minimum, and the winner's index comes back by ballot+shuffle.
//
// k_distinctive: one wave per MapPoint.  Lane i takes observation i and finds the
// median of its distance row by binary search on the value (9 counting passes), then
// the wave takes the smallest (median, i).
#include <hip/hip_runtime.h>

#include "orbx_kernels.h"

namespace orbx {
namespace {

__device__ __forceinline__ unsigned umin32(unsigned a, unsigned b) { return a < b ? a : b; }

__device__ __forceinline__ unsigned row_min16_u32(unsigned v) {
    v = umin32(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
    v = umin32(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
    v = umin32(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
    v = umin32(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
    return v;
}

__device__ __forceinline__ int ham32(const unsigned long long* a, const uint8_t* b) {
    const unsigned long long* q = (const unsigned long long*)b;
    return __popcll(a[0] ^ q[0]) + __popcll(a[1] ^ q[1]) + __popcll(a[2] ^ q[2]) + __popcll(a[3] ^ q[3]);
}

}  // namespace

__global__ __launch_bounds__(256) void k_window_best(const BestProblem* __restrict__ probs) {
    const BestProblem& pb = probs[0];
    const int row = blockIdx.x * 16 + (threadIdx.x >> 4);
    const int sub = threadIdx.x & 15;
    const int rowbase = threadIdx.x & 48;  // lane of the row's first thread within the wave
    if (blockIdx.x * 16 >= pb.nq) return;
    const bool live = row < pb.nq;
    const BestQuery Q = pb.q[live ? row : 0];
    const unsigned long long* qd = (const unsigned long long*)(pb.qdesc + (size_t)(live ? row : 0) * 32);
    const unsigned long long d[4] = {qd[0], qd[1], qd[2], qd[3]};
    // Frame/KeyFrame::GetFeaturesInArea cells (Frame.cc:495-515)
    int t = (int)floorf((Q.u - pb.min_x - Q.r) * pb.inv_w);
    const int x0 = t > 0 ? t : 0;
    t = (int)ceilf((Q.u - pb.min_x + Q.r) * pb.inv_w);
    const int x1 = t < kGridCols - 1 ? t : kGridCols - 1;
    t = (int)floorf((Q.v - pb.min_y - Q.r) * pb.inv_h);
    const int y0 = t > 0 ? t : 0;
    t = (int)ceilf((Q.v - pb.min_y + Q.r) * pb.inv_h);
    const int y1 = t < kGridRows - 1 ? t : kGridRows - 1;
    unsigned best = 0xffffffffu;
    int best_idx = -1;
    if (live && !(x0 >= kGridCols || x1 < 0 || y0 >= kGridRows || y1 < 0)) {
        int rank0 = 0;
        for (int ix = x0; ix <= x1; ix++) {
            const int a = pb.cell_start[ix * kGridRows + y0], b = pb.cell_start[ix * kGridRows + y1 + 1];
            for (int p = a + sub; p < b; p += 16) {
                const int idx = pb.cell_idx[p];
                const orbx_keypoint kp = pb.keys[idx];
                const float distx = kp.x - Q.u, disty = kp.y - Q.v;
                if (!(fabsf(distx) < Q.r && fabsf(disty) < Q.r)) continue;
                const int lv = kp.octave;
                if (lv < Q.pred - 1 || lv > Q.pred) continue;
                if (pb.gate) {
                    float e2;
                    if (pb.u_right && pb.u_right[idx] >= 0) {
                        const float ex = __fsub_rn(Q.u, kp.x), ey = __fsub_rn(Q.v, kp.y),
                                    er = __fsub_rn(Q.ur, pb.u_right[idx]);
                        // fused like the reference's build (H4): fma(er, er, fma(ex, ex, ey*ey))
                        e2 = __fmaf_rn(er, er, __fmaf_rn(ex, ex, __fmul_rn(ey, ey)));
                        if ((double)__fmul_rn(e2, pb.inv_sigma2[lv]) > 7.8) continue;
                    } else {
                        const float ex = __fsub_rn(Q.u, kp.x), ey = __fsub_rn(Q.v, kp.y);
                        e2 = __fmaf_rn(ex, ex, __fmul_rn(ey, ey));
                        if ((double)__fmul_rn(e2, pb.inv_sigma2[lv]) > 5.99) continue;
                    }
                }
                const int dist = ham32(d, pb.desc + (size_t)idx * 32);
                const unsigned key = (unsigned)dist << 23 | (unsigned)(rank0 + p - a);
                if (key < best) {
                    best = key;
                    best_idx = idx;
                }
            }
            rank0 += b - a;
        }
    }
    const unsigned m = row_min16_u32(best);
    const unsigned long long bal = __ballot(best == m);
    const int src = rowbase + __builtin_ctzll((bal >> rowbase) & 0xffffull | (1ull << 16));
    const int idx = __shfl(best_idx, src, 64);
    if (live && sub == 0) pb.best[row] = (m != 0xffffffffu && (int)(m >> 23) <= pb.accept) ? idx : -1;
}

hipError_t launch_window_best(const BestProblem* d_prob, int nq, hipStream_t stream) {
    if (nq <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_window_best, dim3((nq + 15) / 16), dim3(256), 0, stream, d_prob);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_distinctive(int nmp, const int32_t* __restrict__ off,
                                                     const uint8_t* __restrict__ desc, int32_t* __restrict__ best,
                                                     uint8_t* __restrict__ out_desc) {
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (m >= nmp) return;
    const int beg = off[m], N = off[m + 1] - beg;
    if (N <= 0) {
        if (lane == 0) best[m] = -1;
        return;
    }
    const uint8_t* D = desc + (size_t)beg * 32;
    const int k = (int)(0.5 * (double)(N - 1));  // vDists[0.5 * (N - 1)]
    unsigned long long wbest = ~0ull;
    for (int i0 = 0; i0 < N; i0 += 64) {
        const int i = i0 + lane;
        unsigned long long key = ~0ull;
        if (i < N) {
            const unsigned long long* di = (const unsigned long long*)(D + (size_t)i * 32);
            const unsigned long long a[4] = {di[0], di[1], di[2], di[3]};
            // k-th smallest of row i (self distance 0 included): smallest v with
            // #{j : d_ij <= v} >= k + 1
            int lo = 0, hi = 256;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                int cnt = 0;
                for (int j = 0; j < N; j++) cnt += (j == i ? 0 : ham32(a, D + (size_t)j * 32)) <= mid;
                if (cnt >= k + 1)
                    hi = mid;
                else
                    lo = mid + 1;
            }
            key = (unsigned long long)lo << 32 | (unsigned)i;
        }
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long w = (unsigned long long)(unsigned)__shfl_xor((int)(key >> 32), o, 64) << 32 |
                                         (unsigned)__shfl_xor((int)(unsigned)key, o, 64);
            key = w < key ? w : key;
        }
        wbest = key < wbest ? key : wbest;
    }
    const int bi = (int)(unsigned)wbest;
    if (lane == 0) best[m] = bi;
    if (out_desc && lane < 8)
        ((uint32_t*)(out_desc + (size_t)m * 32))[lane] = ((const uint32_t*)(D + (size_t)bi * 32))[lane];
}

hipError_t launch_distinctive(int nmp, const int32_t* off, const uint8_t* desc, int32_t* best, uint8_t* out_desc,
                              hipStream_t stream) {
    if (nmp <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_distinctive, dim3((nmp + 3) / 4), dim3(256), 0, stream, nmp, off, desc, best, out_desc);
    return hipGetLastError();
}

}  // namespace orbx
