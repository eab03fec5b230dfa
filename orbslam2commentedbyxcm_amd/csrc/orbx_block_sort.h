// orbx_block_sort.h -- bitonic sort of up to 8192 u64 keys by one 1024-thread
// workgroup (vocabulary frame builder, device grid).  Element e*1024 + t lives in
// register r[e] of thread t; merge distances below 64 stay inside a wave and run as
// lane shuffles (no barrier), the rest run in place in LDS.
#pragma once

#include <hip/hip_runtime.h>

namespace orbx {

constexpr int kSortThreads = 1024;
constexpr int kSortMaxKeys = 8192;
constexpr int kSortPer = kSortMaxKeys / kSortThreads;

__device__ __forceinline__ unsigned long long sort_shfl_xor64(unsigned long long v, int j) {
    const int lo = __shfl_xor((int)(unsigned)v, j, 64), hi = __shfl_xor((int)(unsigned)(v >> 32), j, 64);
    return (unsigned long long)(unsigned)hi << 32 | (unsigned)lo;
}

// Register stages of a bitonic merge for distances j <= jtop < 64: new value of
// element i is the min of (i, i^j) when "i is the lower index" agrees with "block k
// ascending", else the max.
__device__ __forceinline__ void sort_reg_stages(unsigned long long (&r)[kSortPer], int ne, int k, int jtop) {
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 32; j > 0; j >>= 1) {
        if (j > jtop) continue;
#pragma unroll
        for (int e = 0; e < kSortPer; e++) {
            if (e < ne) {
                const unsigned long long v = r[e], p = sort_shfl_xor64(v, j);
                const int i = e * kSortThreads + t;
                const bool lower = (t & j) == 0, asc = (i & k) == 0;
                r[e] = (lower == asc) ? (v < p ? v : p) : (v < p ? p : v);
            }
        }
    }
}

// Sort m = ne * 1024 keys (ne = 1..8) held in r into s[0, m) ascending.  Ends with the
// sorted keys in s and a barrier.  Must be called by all 1024 threads.
__device__ inline void block_bitonic_sort64(unsigned long long (&r)[kSortPer], int ne, unsigned long long* s) {
    const int t = threadIdx.x, m = ne * kSortThreads;
    for (int k = 2; k <= 64; k <<= 1) sort_reg_stages(r, ne, k, k >> 1);
#pragma unroll
    for (int e = 0; e < kSortPer; e++)
        if (e < ne) s[e * kSortThreads + t] = r[e];
    __syncthreads();
    for (int k = 128; k <= m; k <<= 1) {
        for (int j = k >> 1; j >= 64; j >>= 1) {
            for (int q = t; q < m / 2; q += kSortThreads) {
                const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1));
                const unsigned long long a = s[i], c = s[i + j];
                if ((a > c) == ((i & k) == 0)) {
                    s[i] = c;
                    s[i + j] = a;
                }
            }
            __syncthreads();
        }
#pragma unroll
        for (int e = 0; e < kSortPer; e++)
            if (e < ne) r[e] = s[e * kSortThreads + t];
        sort_reg_stages(r, ne, k, 32);
#pragma unroll
        for (int e = 0; e < kSortPer; e++)
            if (e < ne) s[e * kSortThreads + t] = r[e];
        __syncthreads();
    }
}

}  // namespace orbx
