// orbx_match.hip -- Hamming matching kernels (ORBmatcher hot loops) for gfx950.
//
// DescriptorDistance (ORBmatcher.cc:1983-2003) is a 256-bit XOR + popcount; here it is
// four 64-bit loads, XORs and v_bcnt per descriptor pair.  The candidate scoring of
// SearchByProjection (ORBmatcher.cc:61-173, 1620-1789, 1792-1924) and
// SearchForTriangulation (ORBmatcher.cc:850-1056) is one wave per query: lanes stride
// the query's candidate list and a wave reduction keeps the best and second-best
// (distance, list position) keys, which reproduces the reference's sequential
// `dist < bestDist` / `else if (dist < bestDist2)` updates exactly.
#include <hip/hip_runtime.h>

#include "orbx_kernels.h"

namespace orbx {

__device__ __forceinline__ int hamming32(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b) {
    const unsigned long long* pa = (const unsigned long long*)a;
    const unsigned long long* pb = (const unsigned long long*)b;
    return __popcll(pa[0] ^ pb[0]) + __popcll(pa[1] ^ pb[1]) + __popcll(pa[2] ^ pb[2]) +
           __popcll(pa[3] ^ pb[3]);
}

// 64 x 64 output tile per 256-thread workgroup; descriptors staged through LDS.
__global__ __launch_bounds__(256) void k_hamming_matrix(const uint8_t* __restrict__ a, int na,
                                                        const uint8_t* __restrict__ b, int nb,
                                                        int32_t* __restrict__ dist) {
    __shared__ unsigned long long sa[64][4];
    __shared__ unsigned long long sb[64][4];
    const int tid = threadIdx.x;
    const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
    {
        const int r = tid >> 2, w = tid & 3;
        const int i = i0 + r, j = j0 + r;
        sa[r][w] = i < na ? ((const unsigned long long*)(a + (size_t)i * 32))[w] : 0ull;
        sb[r][w] = j < nb ? ((const unsigned long long*)(b + (size_t)j * 32))[w] : 0ull;
    }
    __syncthreads();
    const int jj = tid & 63;
    const unsigned long long b0 = sb[jj][0], b1 = sb[jj][1], b2 = sb[jj][2], b3 = sb[jj][3];
    for (int ii = tid >> 6; ii < 64; ii += 4) {
        const int i = i0 + ii, j = j0 + jj;
        if (i < na && j < nb) {
            dist[(size_t)i * nb + j] = __popcll(sa[ii][0] ^ b0) + __popcll(sa[ii][1] ^ b1) +
                                       __popcll(sa[ii][2] ^ b2) + __popcll(sa[ii][3] ^ b3);
        }
    }
}

// key = dist << 23 | position (tie_last=0: lowest position wins) or
//       dist << 23 | (0x7fffff - position) (tie_last=1: highest position wins); dist <= 256
__device__ __forceinline__ unsigned make_key(int dist, int pos, int tie_last) {
    return ((unsigned)dist << 23) | (unsigned)(tie_last ? (0x7fffff - pos) : pos);
}

__global__ __launch_bounds__(256) void k_window_match(const uint8_t* __restrict__ qdesc, int nq,
                                                      const uint8_t* __restrict__ tdesc,
                                                      const int32_t* __restrict__ tlevel,
                                                      const int32_t* __restrict__ cand_off,
                                                      const int32_t* __restrict__ cand, int tie_last,
                                                      int32_t* __restrict__ best_idx,
                                                      int32_t* __restrict__ best_dist,
                                                      int32_t* __restrict__ best_level,
                                                      int32_t* __restrict__ second_dist,
                                                      int32_t* __restrict__ second_level) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = blockIdx.x * 4 + wave;
    if (q >= nq) return;
    const unsigned long long* qp = (const unsigned long long*)(qdesc + (size_t)q * 32);
    const unsigned long long q0 = qp[0], q1 = qp[1], q2 = qp[2], q3 = qp[3];
    const int beg = cand_off[q], end = cand_off[q + 1];
    unsigned k1 = 0xffffffffu, k2 = 0xffffffffu;  // best and second keys held by this lane
    for (int p = beg + lane; p < end; p += 64) {
        const int t = cand[p];
        const unsigned long long* tp = (const unsigned long long*)(tdesc + (size_t)t * 32);
        const int d = __popcll(q0 ^ tp[0]) + __popcll(q1 ^ tp[1]) + __popcll(q2 ^ tp[2]) + __popcll(q3 ^ tp[3]);
        const unsigned k = make_key(d, p - beg, tie_last);
        if (k < k1) { k2 = k1; k1 = k; }
        else if (k < k2) { k2 = k; }
    }
    // wave top-2 reduction
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned o1 = __shfl_xor(k1, o), o2 = __shfl_xor(k2, o);
        const unsigned n1 = k1 < o1 ? k1 : o1;
        const unsigned hi = k1 < o1 ? o1 : k1;          // loser of the two bests
        const unsigned lo2 = k2 < o2 ? k2 : o2;         // best of the two seconds
        k1 = n1;
        k2 = hi < lo2 ? hi : lo2;
    }
    if (lane == 0) {
        if (k1 == 0xffffffffu) {
            best_idx[q] = -1;
            best_dist[q] = 256;
            best_level[q] = -1;
        } else {
            const int pos1 = tie_last ? 0x7fffff - (int)(k1 & 0x7fffff) : (int)(k1 & 0x7fffff);
            const int t1 = cand[beg + pos1];
            best_idx[q] = t1;
            best_dist[q] = (int)(k1 >> 23);
            best_level[q] = tlevel ? tlevel[t1] : -1;
        }
        if (k2 == 0xffffffffu) {
            second_dist[q] = 256;
            second_level[q] = -1;
        } else {
            const int pos2 = tie_last ? 0x7fffff - (int)(k2 & 0x7fffff) : (int)(k2 & 0x7fffff);
            const int t2 = cand[beg + pos2];
            second_dist[q] = (int)(k2 >> 23);
            second_level[q] = tlevel ? tlevel[t2] : -1;
        }
    }
}

hipError_t launch_hamming_matrix(const uint8_t* a, int na, const uint8_t* b, int nb, int32_t* dist,
                                 hipStream_t stream) {
    if (na <= 0 || nb <= 0) return hipSuccess;
    dim3 grid((nb + 63) / 64, (na + 63) / 64);
    hipLaunchKernelGGL(k_hamming_matrix, grid, dim3(256), 0, stream, a, na, b, nb, dist);
    return hipGetLastError();
}

hipError_t launch_window_match(const uint8_t* qdesc, int nq, const uint8_t* tdesc, const int32_t* tlevel,
                               const int32_t* cand_off, const int32_t* cand, int tie_last,
                               int32_t* best_idx, int32_t* best_dist, int32_t* best_level,
                               int32_t* second_dist, int32_t* second_level, hipStream_t stream) {
    if (nq <= 0) return hipSuccess;
    dim3 grid((nq + 3) / 4);
    hipLaunchKernelGGL(k_window_match, grid, dim3(256), 0, stream, qdesc, nq, tdesc, tlevel, cand_off, cand,
                       tie_last, best_idx, best_dist, best_level, second_dist, second_level);
    return hipGetLastError();
}

}  // namespace orbx
