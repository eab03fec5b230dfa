// orbx_match.hip -- Hamming matching kernels (ORBmatcher hot loops) for gfx950.
//
// DescriptorDistance (ORBmatcher.cc:1983-2003) is a 256-bit XOR + popcount; here it is
// four 64-bit loads, XORs and v_bcnt per descriptor pair.  The candidate scoring of
// SearchByProjection (ORBmatcher.cc:61-173, 1620-1789, 1792-1924) and
// SearchForTriangulation (ORBmatcher.cc:850-1056) is one wave per query: lanes stride
// the query's candidate list and a wave reduction keeps the best and second-best
// (distance, list position) keys, which reproduces the reference's sequential
// `dist < bestDist` / `else if (dist < bestDist2)` updates exactly.
#include <climits>
#include <hip/hip_runtime.h>

#include <type_traits>

#include "orbx_block_sort.h"
#include "orbx_gmem.h"
#include "orbx_error.h"
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

// Orders a wave's LDS accesses between the steps of a single-wave sequential loop (a
// wave's LDS operations execute in issue order, so this only stops the compiler from
// moving them).  Unlike a workgroup fence it does not wait for the wave's outstanding
// global stores, which would put a memory round trip into every step.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// ------------------------------------------------------------------ projection search

__device__ __forceinline__ bool kp_blocked(int fmp, const ProjParams& P) {
    if (fmp < 0) return false;
    return P.blocked_mode == 1 || P.mp_obs[fmp] > 0;
}

// Claim words: the search's claims (sfmp, the grid's claims) and its queries' MapPoints
// (qmp) carry whether the MapPoint's claim blocks a keypoint as bit 30 (set: it does not,
// a11 / a12's Observations() == 0), so the replay and the re-scoring test a claim with
// one LDS read instead of a dependent Observations() load (MapPoint ids < 2^30, checked
// by the host).  -1: no claim.
constexpr int kClaimFree = 1 << 30;
__device__ __forceinline__ int claim_word(int fmp, const ProjParams& P) {
    return fmp >= 0 && !kp_blocked(fmp, P) ? fmp | kClaimFree : fmp;
}
__device__ __forceinline__ bool claim_blocks(int w) { return w >= 0 && !(w & kClaimFree); }
__device__ __forceinline__ int claim_mp(int w) { return w >= 0 ? w & ~kClaimFree : w; }

struct CellRange {
    int x0, x1, y0, y1;
    bool empty;
};

// Frame::GetFeaturesInArea cell range (Frame.cc:495-515), same float expressions.
__device__ __forceinline__ CellRange cell_range(const ProjProblem& pb, float x, float y, float r) {
    CellRange c;
    int t = (int)floorf((x - pb.min_x - r) * pb.inv_w);
    c.x0 = t > 0 ? t : 0;
    t = (int)ceilf((x - pb.min_x + r) * pb.inv_w);
    c.x1 = t < kGridCols - 1 ? t : kGridCols - 1;
    t = (int)floorf((y - pb.min_y - r) * pb.inv_h);
    c.y0 = t > 0 ? t : 0;
    t = (int)ceilf((y - pb.min_y + r) * pb.inv_h);
    c.y1 = t < kGridRows - 1 ? t : kGridRows - 1;
    c.empty = c.x0 >= kGridCols || c.x1 < 0 || c.y0 >= kGridRows || c.y1 < 0;
    return c;
}

constexpr int kXcds = 8;  // MI355X: 8 XCDs, workgroups dealt round robin, one L2 each
constexpr unsigned kNoKey32 = 0xffffffffu;
constexpr unsigned long long kNoKey = ~0ull;
constexpr int kNoCell = 0xfff;
constexpr int kNumCells = kGridCols * kGridRows;

// The frame's keypoints sorted by (grid cell, index) -- Frame::mGrid flattened, cell
// c = ix*FRAME_GRID_ROWS + iy.  GetFeaturesInArea walks cells ix ascending, iy
// ascending, index ascending, so a keypoint's sorted position is its rank in the
// reference's iteration order; candidate keys (distance << 13 | position) therefore
// order ties exactly as the reference's strict `<` updates do, whatever order the
// lanes visit the candidates in.  The per-keypoint state the scans read (position,
// claim, descriptor) is kept in sorted order.
//
// Octave runs.  Every projection search filters candidates by octave (a window of 1-3
// levels around the predicted one) and the window radius grows with the octave
// (th * scale[level]): at 5000 features x 12 levels a top-level window covers ~800
// keypoints of which ~5 % are in the level range.  So the scan does not walk cells: a
// grid column's keypoints are also listed bucketed by (octave, block of kRowBlk grid rows)
// -- orun, u16 entries position | (iy % kRowBlk) << 13 -- with bucket starts in bstart,
// [ix][octave][block] (+ one sentinel).  A query visits, per column of its window and
// per octave of its range, the buckets of the blocks its rows touch, and drops the rows
// of the two end blocks outside the window (iy % kRowBlk in the entry).  Octaves >= noct share
// the last bucket (the host sets noct above every keypoint's octave).
#ifndef ORBX_ROWBLK_LOG2
// 4-row blocks (round 3): the end blocks of a small window carry fewer rows outside it.
// Scoring alone configs[4] 707 -> 659 us, configs[1] 71.7 -> 66.8 us; 2-row blocks
// 639 / 66.1 us but a slower sort and no pipelined gain (configs[4] 92.6-94.8k against
// 95.4-95.8k frames/s for 4 rows, 93.9-95.4k for 8)
#define ORBX_ROWBLK_LOG2 2
#endif
constexpr int kRowBlkLog2 = ORBX_ROWBLK_LOG2;
constexpr int kRowBlk = 1 << kRowBlkLog2;     // grid rows per bucket block
constexpr int kNumBlk = kGridRows / kRowBlk;  // 6
static_assert(kGridRows % kRowBlk == 0 && kRowBlk <= 8, "row blocks tile the grid; 3 row bits in an orun entry");
__host__ __device__ constexpr int bucket_table_len(int noct) { return kGridCols * noct * kNumBlk + 1; }

struct SortedGrid {
    const unsigned* skey;     // (cell << 18) | (index << 5) | octave, ascending; bit 31: see kKeyBlocked
    const uint16_t* bstart;   // bucket starts into orun, [ix][octave][block], + sentinel
    const uint16_t* orun;     // sorted positions bucketed by (column, octave, row block)
    const float2* sxy;        // x, y
    const uint4* sdesc;       // 2 x uint4 per keypoint, or null (descriptors read from global)
    int noct;                 // octave buckets per column
};
__device__ __forceinline__ int sk_idx(unsigned k) { return (int)((k >> 5) & 0x1fffu); }
__device__ __forceinline__ int sk_oct(unsigned k) { return (int)(k & 31u); }
// Bit 31 of a sorted key (above every cell, kNoCell included): the keypoint is blocked by
// its claim before the search (kp_blocked).  Set only by the split scoring kernel, which
// then holds no claims array in LDS; the published grid has it cleared.
constexpr unsigned kKeyBlocked = 0x80000000u;

// bucket of the keypoint with sorted key k in grid column ix: octave-major, then block
__device__ __forceinline__ int bucket_of(unsigned k, int ix, int noct) {
    const int iy = (int)(k >> 18) - ix * kGridRows;
    const int o = sk_oct(k) < noct ? sk_oct(k) : noct - 1;
    return o * kNumBlk + (iy >> kRowBlkLog2);
}

// colstart[c] = first sorted position whose grid column is >= c (c = 0..kGridCols;
// off-grid keypoints sort last, so colstart[kGridCols] counts the keypoints in the
// grid).  Each entry is written once.
template <int NT>
__device__ void build_colstart(const unsigned* skey, int n, uint16_t* colstart) {
    for (int p = threadIdx.x; p <= n; p += NT) {
        const int prev = p == 0 ? -1 : min((int)(skey[p - 1] >> 18) / kGridRows, kGridCols);
        const int cur = p == n ? kGridCols : min((int)(skey[p] >> 18) / kGridRows, kGridCols);
        for (int c = prev + 1; c <= cur; c++) colstart[c] = (uint16_t)p;
    }
}

// Inclusive prefix sum over the 64 lanes of a wave (all lanes active): DPP row_shr
// 1/2/4/8 inside each 16-lane row, then row_bcast:15 and row_bcast:31 across rows.
__device__ __forceinline__ unsigned wave_inclusive_sum(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}

// LDS scratch of build_octave_runs: one u32 counter per bucket
__host__ __device__ constexpr size_t octave_runs_scratch(int noct) {
    return (size_t)kGridCols * noct * kNumBlk * 4;
}

// The octave runs of a sorted grid (after build_colstart and a barrier): LDS counters
// per bucket, one wave-scan per column from colstart[ix] for the bucket starts, then
// every keypoint takes a slot of its bucket.  Slots inside a bucket come in atomic
// order: the scan's result does not depend on the order it visits candidates in (keys
// carry the sorted position).  cnt: octave_runs_scratch(noct) bytes of LDS.  Whole
// workgroup; the caller puts a barrier after it.
template <int NT>
__device__ void build_octave_runs(const unsigned* skey, const uint16_t* colstart, int noct, uint16_t* bstart,
                                  uint16_t* orun, unsigned* cnt) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kW = NT / 64;
    const int nb = noct * kNumBlk, nt = kGridCols * nb, ng = colstart[kGridCols];
    for (int t = tid; t < nt; t += NT) cnt[t] = 0u;
    __syncthreads();
    for (int p = tid; p < ng; p += NT) {
        const unsigned k = skey[p];
        const int ix = (int)(k >> 18) / kGridRows;
        atomicAdd(&cnt[ix * nb + bucket_of(k, ix, noct)], 1u);
    }
    __syncthreads();
    constexpr int kMaxPer = (32 * kNumBlk + 63) / 64;  // noct <= 32
    const int per = (nb + 63) >> 6;  // consecutive buckets per lane, <= kMaxPer
    for (int ix = wave; ix < kGridCols; ix += kW) {
        unsigned v[kMaxPer], sum = 0;
#pragma unroll
        for (int j = 0; j < kMaxPer; j++) {
            const int u = lane * per + j;
            v[j] = (j < per && u < nb) ? cnt[ix * nb + u] : 0u;
            sum += v[j];
        }
        unsigned run = colstart[ix] + wave_inclusive_sum(sum) - sum;
#pragma unroll
        for (int j = 0; j < kMaxPer; j++) {
            const int u = lane * per + j;
            if (j < per && u < nb) {
                cnt[ix * nb + u] = run;
                bstart[ix * nb + u] = (uint16_t)run;
                run += v[j];
            }
        }
    }
    if (tid == 0) bstart[nt] = (uint16_t)ng;
    __syncthreads();
    for (int p = tid; p < ng; p += NT) {
        const unsigned k = skey[p];
        const int ix = (int)(k >> 18) / kGridRows, iy = (int)(k >> 18) - ix * kGridRows;
        const unsigned slot = atomicAdd(&cnt[ix * nb + bucket_of(k, ix, noct)], 1u);
        orun[slot] = (uint16_t)(p | ((iy & (kRowBlk - 1)) << 13));  // 3 bits: kRowBlk <= 8
    }
}

constexpr int kProjThreads = 1024;      // default workgroup size of k_proj_search
constexpr int kProjThreadsSmall = 256;  // small-footprint variant (overlapped with other work)
constexpr int kProjThreadsTiny = 64;    // one wave per problem (a background stream's footprint)
#ifndef ORBX_SPLIT_SCORE_THREADS
#define ORBX_SPLIT_SCORE_THREADS 1024
#endif
// the sequence matcher's scoring workgroup (r05w: 512 threads within noise at configs[1],
// configs[4] 113.6-115.4k -> 106.1-107.0k frames/s)
constexpr int kSplitScoreThreads = ORBX_SPLIT_SCORE_THREADS;
constexpr int kTopK = ORBX_TOPK;
#ifndef ORBX_LANE_TOPK
#define ORBX_LANE_TOPK 6
#endif
// candidates each scoring lane keeps before the group merge.  A lane that saw more and
// runs dry truncates the query's list (a re-scoring on the replay's critical path later):
// 6 measured configs[4] 81.5k frames/s against 77.0k for 4 and 81.0k for 8, configs[1]
// unchanged (profiles/r02_n_lane_topk_ab.log)
constexpr int kLaneTopK = ORBX_LANE_TOPK;           // candidate-list length per query
// The sequence matcher's split scoring kernel runs beside the extraction lanes, where its
// registers are what counts (4 waves a SIMD: every VGPR it holds is 4 the extraction's waves
// on that SIMD cannot have).  Without the next-query prefetch it holds 83 VGPRs instead of
// 102 and 80 with lane lists of 4: RGB-D configs[4] 88.3-88.4k -> 89.3-89.5k (no prefetch)
// -> 90.6-91.0k frames/s (lists of 4; 3 and 5 measured 89.8k and 89.3-89.6k), configs[1]
// 228.0-228.8k -> 229.4-230.0k (profiles/r06_scoring_registers_ab.txt).  The single calls
// keep both (their latency is the query loads').
#ifndef ORBX_SPLIT_LANE_TOPK
#define ORBX_SPLIT_LANE_TOPK 4
#endif
#ifndef ORBX_SPLIT_PREFETCH
#define ORBX_SPLIT_PREFETCH 0
#endif
constexpr int kSplitLaneTopK = ORBX_SPLIT_LANE_TOPK;
// Lanes per query of the split scoring (0: by window width, 4 / 8 / 16 as the other forms).
// Two: the balance counters (-DORBX_SCORE_COUNT) showed a 16-lane group's busiest lane with
// twice its mean work and the wave's with 2.5 times, which smaller groups cut; a pair
// merges with one DPP step and keeps lists of 6 per lane.  RGB-D configs[4] 91.8-91.9k (by
// width) -> 94.0-94.2k frames/s; one lane (lists of 12) 84.6-84.8k, four 91.5-91.6k; lists of
// 4 / 5 / 8 for the pair 90.5-90.7k / 91.0-91.5k / 93.1-93.6k against 93.1-93.6k for 6;
// configs[1] 228.9-230.0k -> 230.8-232.5k (profiles/r06_scoring_registers_ab.txt).
#ifndef ORBX_SPLIT_KR_ALL
#define ORBX_SPLIT_KR_ALL 2
#endif
constexpr int kSplitKr = ORBX_SPLIT_KR_ALL;
#ifndef ORBX_SPLIT_KR2_TOPK
#define ORBX_SPLIT_KR2_TOPK 6
#endif
// a lane's list length in a KR-lane group of the split scoring: a lone lane keeps the whole list
__host__ __device__ constexpr int split_lane_topk(int kr) {
    return kr == 1 ? kTopK : kr == 2 ? ORBX_SPLIT_KR2_TOPK : kSplitLaneTopK;
}
static_assert(kTopK % 4 == 0, "lists are stored as uint4s");
constexpr int kListVec = kTopK / 4;        // uint4s per stored list
constexpr int kListWords = kTopK / 2;      // u64 words per stored list
static_assert(kProjScratchWords >= kListWords + 2, "per-query global scratch holds the list, mp + angle, match + bin");
constexpr unsigned kNoEntry = 0xffffffffu;  // no further candidate
constexpr unsigned kTrunc = 0xfffffffeu;    // further candidates exist but are not listed

// Candidate-list entry: distance << 18 | octave << 13 | sorted position.  Entries of a
// query are kept in the reference's (distance, iteration order) order.
__device__ __forceinline__ int ent_dist(unsigned e) { return (int)(e >> 18); }
__device__ __forceinline__ int ent_oct(unsigned e) { return (int)((e >> 13) & 31u); }
__device__ __forceinline__ int ent_pos(unsigned e) { return (int)(e & 0x1fffu); }

// The same over the 4 lanes of each DPP quad (quad_perm [1,0,3,2], [2,3,0,1]).
__device__ __forceinline__ unsigned quad_min_u32(unsigned v);

// Row minimum over the 16 lanes of each DPP row (quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror): every lane of the row ends with the row's minimum.
// Must be called with the whole wave active.
__device__ __forceinline__ unsigned umin_(unsigned a, unsigned b) { return a < b ? a : b; }
__device__ __forceinline__ unsigned row_min_u32(unsigned v) {
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
    return v;
}

// The same over the 8 lanes of each half DPP row (quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror).
__device__ __forceinline__ unsigned half_row_min_u32(unsigned v) {
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
    return v;
}

__device__ __forceinline__ unsigned pair_min_u32(unsigned v) {  // lane pairs: quad_perm [1,0,3,2]
    return umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
}

__device__ __forceinline__ unsigned quad_min_u32(unsigned v) {
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
    return v;
}

// A query and its MapPoint descriptor held in registers (loaded ahead of use so the
// global latency overlaps the LDS work of the previous query).
struct QueryReg {
    ProjQuery q;
    uint4 d0, d1;
};
static_assert(sizeof(ProjQuery) == 48, "ProjQuery layout");

__device__ __forceinline__ QueryReg load_query(const ProjProblem& pb, int q) {
    QueryReg r;
    r.q = ldg(pb.q + q);
    const uint4* d = (const uint4*)(pb.qdesc + (size_t)q * 32);
    r.d0 = ldg(d);
    r.d1 = ldg(d + 1);
    return r;
}

// Lane `src`'s query, broadcast to the whole wave (v_readlane per word).
__device__ __forceinline__ QueryReg bcast_query(const QueryReg& x, int src) {
    constexpr int kW = (int)(sizeof(QueryReg) / 4);
    static_assert(sizeof(QueryReg) % 4 == 0, "QueryReg words");
    int w[kW];
    __builtin_memcpy(w, &x, sizeof(QueryReg));
#pragma unroll
    for (int i = 0; i < kW; i++) w[i] = __builtin_amdgcn_readlane(w[i], src);
    QueryReg r;
    __builtin_memcpy(&r, w, sizeof(QueryReg));
    return r;
}

// Lane `src`'s query for each lane (src may differ per lane; ds_bpermute per word).
__device__ __forceinline__ QueryReg shfl_query(const QueryReg& x, int src) {
    constexpr int kW = (int)(sizeof(QueryReg) / 4);
    int w[kW];
    __builtin_memcpy(w, &x, sizeof(QueryReg));
#pragma unroll
    for (int i = 0; i < kW; i++) w[i] = __shfl(w[i], src);
    QueryReg r;
    __builtin_memcpy(&r, w, sizeof(QueryReg));
    return r;
}

#ifndef ORBX_MED3_INSERT
#define ORBX_MED3_INSERT 1
#endif
// v_med3_u32 (no integer builtin; max(a, min(b, c)) is not matched to it)
__device__ __forceinline__ unsigned med3_u32(unsigned a, unsigned b, unsigned c) {
    unsigned d;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
// Insert key into the ascending list k[0..L) (keys distinct), dropping the largest.  With
// k[i-1] <= k[i] the new k[i] is max(k[i-1], min(key, k[i])) = med3(k[i-1], key, k[i]):
// one instruction per entry, top down, branch-free (a key above k[L-1] changes nothing).
template <int L>
__device__ __forceinline__ void sorted_insert(unsigned (&k)[L], unsigned key) {
#if ORBX_MED3_INSERT
#pragma unroll
    for (int i = L - 1; i > 0; i--) k[i] = med3_u32(k[i - 1], key, k[i]);
    k[0] = key < k[0] ? key : k[0];
#else
    if (key < k[L - 1]) {  // top down (reads k[i-1] first)
#pragma unroll
        for (int i = L - 1; i > 0; i--) k[i] = key < k[i - 1] ? k[i - 1] : (key < k[i] ? key : k[i]);
        k[0] = key < k[0] ? key : k[0];
    }
#endif
}

// The kTopK best candidates of a query (GetFeaturesInArea + the overload's filters)
// against the current claims sfmp, as entries (kNoEntry = no more candidates, kTrunc =
// more candidates exist than listed).  One 16-lane row per query, four queries per wave:
// the row's lanes split the columns of the query's cell window (and the sorted-position
// runs inside them), keep a local top-kLaneTopK of (distance << 13 | position) and merge
// them by DPP row minima.  A lane that saw more candidates only knows its best ones, so the
// merged list is exact up to the point where such a lane runs dry; the rest is kTrunc.
// The candidate windows hold a few to a few tens of keypoints, so a row keeps its lanes
// busy where a whole wave per query would mostly idle.  `valid` false: no query in this
// row (out = kNoEntry).  Must be called with the whole wave active.
// K = 64: one query per wave, all lanes over its window (the replay's re-scoring of a
// query whose list ran out, a single query on the critical path).
#ifndef ORBX_SCORE_KR_FIXED
#define ORBX_SCORE_KR_FIXED 0
#endif
#ifndef ORBX_VISIT_RCP
#define ORBX_VISIT_RCP 1
#endif
#ifndef ORBX_SCORE_PAIR
// two bucket entries per scan step with descriptors from global memory (round 3): the
// configs[4] matcher alone 1.114 -> 1.047 ms, the drop-in rows a11-a14 1-3 % faster,
// pipelined steps unchanged (within noise)
#define ORBX_SCORE_PAIR 1
#endif
template <int K, int KL = kLaneTopK>
__device__ void score_groupk(const ProjProblem& pb, const ProjParams& P, const QueryReg& QR, bool valid,
                             const SortedGrid& G, const int* sfmp, unsigned out[kTopK]) {
    static_assert(K == 1 || K == 2 || K == 4 || K == 8 || K == 16 || K == 64,
                  "a lane, a lane pair, a DPP quad, half a DPP row, a DPP row or a wave");
    const int r = threadIdx.x & (K - 1);
    const ProjQuery& Q = QR.q;
    unsigned k[KL];
#pragma unroll
    for (int i = 0; i < KL; i++) k[i] = kNoEntry;
    int seen = 0;
#if ORBX_SCORE_COUNT
    unsigned long long n_pair = 0, n_step = 0, n_ok = 0;
#endif
    if (valid) {
        const CellRange cr = cell_range(pb, Q.u, Q.v, Q.r);
        if (!cr.empty) {
            const unsigned long long q0 = (unsigned long long)QR.d0.y << 32 | QR.d0.x;
            const unsigned long long q1 = (unsigned long long)QR.d0.w << 32 | QR.d0.z;
            const unsigned long long q2 = (unsigned long long)QR.d1.y << 32 | QR.d1.x;
            const unsigned long long q3 = (unsigned long long)QR.d1.w << 32 | QR.d1.z;
            // the candidates' octave range: GetFeaturesInArea's level filter (applied
            // only when minLevel > 0 || maxLevel >= 0, Frame.cc:515-521) and the
            // overload's own post filter (a14)
            int olo = 0, ohi = 31;
            if ((Q.min_level > 0) || (Q.max_level >= 0)) {
                olo = Q.min_level > 0 ? Q.min_level : 0;
                if (Q.max_level >= 0) ohi = Q.max_level;
            }
            if (Q.post_max >= 0) {
                olo = max(olo, Q.post_min);
                ohi = min(ohi, Q.post_max);
            }
            const int noct = G.noct;
            const int blo = min(olo, noct - 1), bhi = olo > ohi ? -1 : min(ohi, noct - 1);
            const int b0 = cr.y0 >> kRowBlkLog2, b1 = cr.y1 >> kRowBlkLog2;
            const int ylo = cr.y0 & (kRowBlk - 1), yhi = cr.y1 & (kRowBlk - 1);
            const int ncol = cr.x1 - cr.x0 + 1;
            // the (column, octave) visits of the window, octave fastest, dealt over the
            // group's lanes: lanes per visit the most (a power of two) that still cover
            // every visit in one pass; a visit's lanes split its scan.  (Until round 6 the
            // lanes split the columns and each walked every octave of its column: the
            // stereo / RGB-D searches' forward and backward ranges -- up to every level --
            // then left each lane a dozen nearly empty visits.)
            const int nor = bhi - blo + 1;
            const int nv = nor > 0 ? ncol * nor : 0;
            constexpr int kLog2K = K == 1 ? 0 : K == 2 ? 1 : K == 4 ? 2 : (K == 8 ? 3 : (K == 16 ? 4 : 6));
            int sh = 0;
            while (sh < kLog2K && (nv << (sh + 1)) <= K) sh++;
            const int lpc = 1 << sh, sub = r & (lpc - 1);
#if ORBX_VISIT_RCP
            // v / nor without an integer division (~25 VALU): (v + 0.5) / nor lies at least
            // 0.5 / nor >= 1/64 from an integer (nor <= 32, v < 2^11), far above the error of
            // v_rcp_f32 and one multiply
            const float inv_nor = __builtin_amdgcn_rcpf((float)max(nor, 1));
#endif
            for (int v = r >> sh; v < nv; v += K >> sh) {
#if ORBX_VISIT_RCP
                const int cq = (int)(((float)v + 0.5f) * inv_nor);
#else
                const int cq = v / nor;
#endif
                const int ix = cr.x0 + cq, o = blo + (v - cq * nor);
                {
                    // the rows y0..y1 of this column and octave: blocks b0..b1, whose
                    // first / last block also hold rows outside the window
                    const uint16_t* bt = G.bstart + (ix * noct + o) * kNumBlk;
                    const int s0 = bt[b0], e0 = bt[b0 + 1], s1 = bt[b1], e1 = bt[b1 + 1];
#if ORBX_SCORE_COUNT
                    n_pair++;
#endif
#if ORBX_SCORE_PAIR
                    if (!G.sdesc) {
                        // two entries per step (a and a + lpc): their LDS chains (entry,
                        // position, key) and descriptor loads are independent, so they overlap
                        auto test = [&](int a, int ent, float2 kp, unsigned kk, int p) {
                            const int yr = ent >> 13;
                            if ((a < e0 && yr < ylo) || (a >= s1 && yr > yhi)) return false;
                            if (!(fabsf(kp.x - Q.u) < Q.r && fabsf(kp.y - Q.v) < Q.r)) return false;
                            if (sfmp && claim_blocks(sfmp[p])) return false;
                            return (kk & kKeyBlocked) == 0u;
                        };
                        for (int a = s0 + sub; a < e1; a += 2 * lpc) {
                            const int a2 = a + lpc;
                            const bool h2 = a2 < e1;
                            const int entA = G.orun[a], entB = G.orun[h2 ? a2 : a];
                            const int pA = entA & 0x1fff, pB = entB & 0x1fff;
                            const float2 kA = G.sxy[pA], kB = G.sxy[pB];
                            const unsigned kkA = G.skey[pA], kkB = G.skey[pB];
                            const bool okA = test(a, entA, kA, kkA, pA);
                            const bool okB = h2 && test(a2, entB, kB, kkB, pB);
#if ORBX_SCORE_COUNT
                            n_step++;
                            n_ok += (okA ? 1 : 0) + (okB ? 1 : 0);
#endif
                            if (!okA && !okB) continue;
                            const int iA = sk_idx(kkA), iB = sk_idx(okB ? kkB : kkA);
                            const ulonglong2* tA = (const ulonglong2*)(pb.desc + (size_t)iA * 32);
                            const ulonglong2* tB = (const ulonglong2*)(pb.desc + (size_t)iB * 32);
                            const ulonglong2 yA0 = ldg(tA), yA1 = ldg(tA + 1), yB0 = ldg(tB), yB1 = ldg(tB + 1);
                            const unsigned long long xA0 = yA0.x, xA1 = yA0.y, xA2 = yA1.x, xA3 = yA1.y;
                            const unsigned long long xB0 = yB0.x, xB1 = yB0.y, xB2 = yB1.x, xB3 = yB1.y;
                            float urA = 0.f, urB = 0.f;
                            if (Q.er_max >= 0.f && pb.u_right) {
                                urA = ldg(pb.u_right + iA);
                                urB = ldg(pb.u_right + iB);
                            }
                            auto take = [&](bool ok, float ur, int p, unsigned long long x0, unsigned long long x1,
                                            unsigned long long x2, unsigned long long x3) {
                                if (!ok || (ur > 0 && fabsf(Q.ur - ur) > Q.er_max)) return;
                                const int d = __popcll(q0 ^ x0) + __popcll(q1 ^ x1) + __popcll(q2 ^ x2) + __popcll(q3 ^ x3);
                                const unsigned key = ((unsigned)d << 13) | (unsigned)p;
                                seen++;
                                sorted_insert<KL>(k, key);
                            };
                            take(okA, urA, pA, xA0, xA1, xA2, xA3);
                            take(okB, urB, pB, xB0, xB1, xB2, xB3);
                        }
                        continue;
                    }
#endif
                    for (int a = s0 + sub; a < e1; a += lpc) {
                        const int ent = G.orun[a];
                        const int p = ent & 0x1fff, yr = ent >> 13;
                        if ((a < e0 && yr < ylo) || (a >= s1 && yr > yhi)) continue;
                        const float2 kp = G.sxy[p];
                        const float distx = kp.x - Q.u;
                        const float disty = kp.y - Q.v;
                        if (!(fabsf(distx) < Q.r && fabsf(disty) < Q.r)) continue;
                        if (sfmp && claim_blocks(sfmp[p])) continue;  // null: nothing claimed yet
                        int d;
                        if (G.sdesc) {
                            if (Q.er_max >= 0.f && pb.u_right) {
                                const float ur = ldg(pb.u_right + sk_idx(G.skey[p]));
                                if (ur > 0 && fabsf(Q.ur - ur) > Q.er_max) continue;
                            }
                            const uint4 a4 = G.sdesc[2 * p], b4 = G.sdesc[2 * p + 1];
                            d = __popcll(q0 ^ ((unsigned long long)a4.y << 32 | a4.x)) +
                                __popcll(q1 ^ ((unsigned long long)a4.w << 32 | a4.z)) +
                                __popcll(q2 ^ ((unsigned long long)b4.y << 32 | b4.x)) +
                                __popcll(q3 ^ ((unsigned long long)b4.w << 32 | b4.z));
                        } else {
                            const unsigned kk = G.skey[p];
                            if (kk & kKeyBlocked) continue;
                            const int i = sk_idx(kk);
                            if (Q.er_max >= 0.f && pb.u_right) {
                                const float ur = ldg(pb.u_right + i);
                                if (ur > 0 && fabsf(Q.ur - ur) > Q.er_max) continue;
                            }
                            const ulonglong2* tt = (const ulonglong2*)(pb.desc + (size_t)i * 32);
                            const ulonglong2 t0 = ldg(tt), t1 = ldg(tt + 1);
                            d = __popcll(q0 ^ t0.x) + __popcll(q1 ^ t0.y) + __popcll(q2 ^ t1.x) + __popcll(q3 ^ t1.y);
                        }
                        const unsigned key = ((unsigned)d << 13) | (unsigned)p;
                        seen++;
                        sorted_insert<KL>(k, key);
                    }
                }
            }
        }
    }
#if ORBX_SCORE_COUNT
    // balance: a lane's work (visits + scan steps), its group's maximum and its wave's
    int gmax = valid ? (int)(n_pair + n_step) : 0;
    for (int o = K / 2; o > 0; o >>= 1) gmax = max(gmax, __shfl_xor(gmax, o));
    int wmax = gmax;
    for (int o = 32; o >= K; o >>= 1) wmax = max(wmax, __shfl_xor(wmax, o));
    if (P.stamps && valid) {
        unsigned long long* sc = P.stamps + kStampWords * (size_t)blockIdx.x;
        atomicAdd(sc + kStampScore, n_pair);
        atomicAdd(sc + kStampScore + 1, n_step);
        atomicAdd(sc + kStampScore + 2, n_ok);
        if (r == 0) {
            atomicAdd(sc + kStampScore + 3, 1ull);
            atomicAdd(sc + kStampScore + 4, (unsigned long long)gmax);
            atomicAdd(sc + kStampScore + 5, (unsigned long long)wmax);
        }
    }
#endif
    // Group top-kTopK: keys are unique (distinct positions), so one lane pops each minimum.
    const int rsh = K == 64 ? 0 : (threadIdx.x & (63 & ~(K - 1)));  // first lane of this group
    const unsigned long long gmask = K == 64 ? ~0ull : ((1ull << K) - 1);
    bool over = seen > KL;
    bool trunc = false;
    unsigned m[kTopK];
#pragma unroll
    for (int j = 0; j < kTopK; j++) {
        // a lane whose listed candidates are used up but that saw more makes the rest unknown
        const unsigned long long dry = __ballot(over && k[0] == kNoEntry);
        trunc = trunc || ((dry >> rsh) & gmask) != 0;
        m[j] = K == 1   ? k[0]
               : K == 2 ? pair_min_u32(k[0])
               : K == 4 ? quad_min_u32(k[0])
                        : (K == 8 ? half_row_min_u32(k[0]) : row_min_u32(k[0]));
        if (K == 64) {  // the four rows' minima by v_readlane: wave-uniform, no LDS round trip
            m[j] = umin_(umin_((unsigned)__builtin_amdgcn_readlane((int)m[j], 0),
                               (unsigned)__builtin_amdgcn_readlane((int)m[j], 16)),
                         umin_((unsigned)__builtin_amdgcn_readlane((int)m[j], 32),
                               (unsigned)__builtin_amdgcn_readlane((int)m[j], 48)));
        }
        if (k[0] == m[j] && m[j] != kNoEntry) {
#pragma unroll
            for (int i = 0; i < KL - 1; i++) k[i] = k[i + 1];
            k[KL - 1] = kNoEntry;
        }
        if (trunc) m[j] = kTrunc;
    }
#pragma unroll
    for (int j = 0; j < kTopK; j++)
        out[j] = m[j] >= kTrunc ? m[j]
                                : ((m[j] >> 13) << 18) | ((unsigned)sk_oct(G.skey[m[j] & 0x1fffu]) << 13) |
                                      (m[j] & 0x1fffu);
}

constexpr int kScoreRow = 16;  // lanes per query of k_seq_score
__device__ __forceinline__ void score_rowk(const ProjProblem& pb, const ProjParams& P, const QueryReg& QR, bool valid,
                                           const SortedGrid& G, const int* sfmp, unsigned out[kTopK]) {
    score_groupk<kScoreRow>(pb, P, QR, valid, G, sfmp, out);
}

#ifndef ORBX_SPLIT_PERSIST
#define ORBX_SPLIT_PERSIST 1
#endif
#ifndef ORBX_PERSIST_BATCH
#define ORBX_PERSIST_BATCH 32
#endif
// The split scoring's lane pairs without lockstep between pairs (ORBX_SPLIT_PERSIST): a pair
// walks its query's visits and scans as score_groupk<2> does, and when both its lanes are
// through it merges, writes the list and takes the workgroup's next query from an LDS
// counter.  In lockstep a wave's 32 pairs wait for the busiest on every query (1.4 times
// the mean work, -DORBX_SCORE_COUNT); here a wave's iteration is one visit step and one
// scan step of every lane with work.  Merges, list writes and query loads run for
// kPersistBatch lanes at a time (or when no lane is left scanning), so that block runs once
// per several queries.  Same lists as score_groupk<2>.
constexpr int kPersistBatch = ORBX_PERSIST_BATCH;
__device__ void score_pairs(const ProjProblem& pb, const ProjParams& P, const SortedGrid& G, uint4* qk, int* qmp,
                            float* qang, int* s_next) {
    constexpr int KL = split_lane_topk(2);
    const int nq = pb.nq, noct = G.noct;
    const int lane = threadIdx.x & 63, r = lane & 1;
    int q = -1;  // current query; >= nq: retired
    bool fresh = true;
    unsigned long long q0 = 0, q1 = 0, q2 = 0, q3 = 0;
    float qu = 0.f, qv = 0.f, qr = 0.f, qur = 0.f, qer = -1.f, ang = 0.f;
    int mp = -1;
    int x0 = 0, nor = 1, nv = 0, blo = 0, b0 = 0, b1 = 0, ylo = 0, yhi = 0, v = 0, vstep = 2, sub = 0, lpc = 1;
    float inv_nor = 1.f;
    int a = 0, e0 = 0, s1 = 0, e1 = 0;
    unsigned k[KL];
#pragma unroll
    for (int i = 0; i < KL; i++) k[i] = kNoEntry;
    int seen = 0;
    const bool ur_check = pb.u_right != nullptr;
    while (true) {
        const bool ldone = !fresh && q < nq && v >= nv && a >= e1;
        const bool pdone = ldone && __builtin_amdgcn_update_dpp(0, (int)ldone, 0xB1, 0xF, 0xF, false) != 0;
        const bool want = fresh || pdone;
        const unsigned long long wm = __ballot(want), busy = __ballot(!want && q < nq);
        if (__popcll(wm) >= kPersistBatch || busy == 0) {
            // the pairs' merges (score_groupk's, on copies: the other pairs keep scanning)
            unsigned c[KL];
#pragma unroll
            for (int i = 0; i < KL; i++) c[i] = k[i];
            const bool over = seen > KL;
            bool trunc = false;
            unsigned m[kTopK];
#pragma unroll
            for (int j = 0; j < kTopK; j++) {
                const unsigned long long dry = __ballot(over && c[0] == kNoEntry);
                trunc = trunc || ((dry >> (lane & ~1)) & 3ull) != 0;
                m[j] = pair_min_u32(c[0]);
                if (c[0] == m[j] && m[j] != kNoEntry) {
#pragma unroll
                    for (int i = 0; i < KL - 1; i++) c[i] = c[i + 1];
                    c[KL - 1] = kNoEntry;
                }
                if (trunc) m[j] = kTrunc;
            }
            if (pdone && r == 0) {
#pragma unroll
                for (int j = 0; j < kTopK; j++)
                    m[j] = m[j] >= kTrunc ? m[j]
                                          : ((m[j] >> 13) << 18) | ((unsigned)sk_oct(G.skey[m[j] & 0x1fffu]) << 13) |
                                                (m[j] & 0x1fffu);
#pragma unroll
                for (int w = 0; w < kListVec; w++)
                    qk[kListVec * q + w] = make_uint4(m[4 * w], m[4 * w + 1], m[4 * w + 2], m[4 * w + 3]);
                qmp[q] = claim_word(mp, P);
                qang[q] = ang;
            }
            int nqi = 0;
            if (want && r == 0) nqi = atomicAdd(s_next, 1);
            nqi = __builtin_amdgcn_update_dpp(0, nqi, 0xA0, 0xF, 0xF, false);  // the pair's first lane's
            if (want) {
                q = nqi;
                fresh = false;
                nv = 0;
                v = 0;
                a = e1 = 0;
                seen = 0;
#pragma unroll
                for (int i = 0; i < KL; i++) k[i] = kNoEntry;
                if (q < nq) {
                    const QueryReg QR = load_query(pb, q);
                    const ProjQuery& Q = QR.q;
                    mp = Q.mp;
                    ang = Q.angle;
                    qu = Q.u, qv = Q.v, qr = Q.r, qur = Q.ur, qer = Q.er_max;
                    if (mp >= 0) {
                        const CellRange cr = cell_range(pb, Q.u, Q.v, Q.r);
                        if (!cr.empty) {
                            q0 = (unsigned long long)QR.d0.y << 32 | QR.d0.x;
                            q1 = (unsigned long long)QR.d0.w << 32 | QR.d0.z;
                            q2 = (unsigned long long)QR.d1.y << 32 | QR.d1.x;
                            q3 = (unsigned long long)QR.d1.w << 32 | QR.d1.z;
                            int olo = 0, ohi = 31;  // the octave range, as score_groupk
                            if ((Q.min_level > 0) || (Q.max_level >= 0)) {
                                olo = Q.min_level > 0 ? Q.min_level : 0;
                                if (Q.max_level >= 0) ohi = Q.max_level;
                            }
                            if (Q.post_max >= 0) {
                                olo = max(olo, Q.post_min);
                                ohi = min(ohi, Q.post_max);
                            }
                            blo = min(olo, noct - 1);
                            const int bhi = olo > ohi ? -1 : min(ohi, noct - 1);
                            b0 = cr.y0 >> kRowBlkLog2, b1 = cr.y1 >> kRowBlkLog2;
                            ylo = cr.y0 & (kRowBlk - 1), yhi = cr.y1 & (kRowBlk - 1);
                            x0 = cr.x0;
                            nor = bhi - blo + 1;
                            nv = nor > 0 ? (cr.x1 - cr.x0 + 1) * nor : 0;
                            inv_nor = __builtin_amdgcn_rcpf((float)max(nor, 1));
                            const int sh = nv <= 1 ? 1 : 0;  // score_groupk<2>'s lanes per visit
                            lpc = 1 << sh, sub = r & (lpc - 1), v = r >> sh, vstep = 2 >> sh;
                        }
                    }
                } else {
                    q = nq;
                }
            }
        }
        if (__ballot(q < nq) == 0) break;
        // the next (column, octave) visit of a lane whose scan is through
        if (!fresh && q < nq && a >= e1 && v < nv) {
            const int cq = (int)(((float)v + 0.5f) * inv_nor);
            const int ix = x0 + cq, o = blo + (v - cq * nor);
            const uint16_t* bt = G.bstart + (ix * noct + o) * kNumBlk;
            a = bt[b0] + sub, e0 = bt[b0 + 1], s1 = bt[b1], e1 = bt[b1 + 1];
            v += vstep;
        }
        // one scan step: entries a and a + lpc (score_groupk's pair form)
        if (!fresh && q < nq && a < e1) {
            const int a2 = a + lpc;
            const bool h2 = a2 < e1;
            const int entA = G.orun[a], entB = G.orun[h2 ? a2 : a];
            const int pA = entA & 0x1fff, pB = entB & 0x1fff;
            const float2 kA = G.sxy[pA], kB = G.sxy[pB];
            const unsigned kkA = G.skey[pA], kkB = G.skey[pB];
            auto test = [&](int at, int ent, float2 kp, unsigned kk) {
                const int yr = ent >> 13;
                if ((at < e0 && yr < ylo) || (at >= s1 && yr > yhi)) return false;
                if (!(fabsf(kp.x - qu) < qr && fabsf(kp.y - qv) < qr)) return false;
                return (kk & kKeyBlocked) == 0u;
            };
            const bool okA = test(a, entA, kA, kkA);
            const bool okB = h2 && test(a2, entB, kB, kkB);
            a += 2 * lpc;
            if (okA || okB) {
                const int iA = sk_idx(kkA), iB = sk_idx(okB ? kkB : kkA);
                const ulonglong2* tA = (const ulonglong2*)(pb.desc + (size_t)iA * 32);
                const ulonglong2* tB = (const ulonglong2*)(pb.desc + (size_t)iB * 32);
                const ulonglong2 yA0 = ldg(tA), yA1 = ldg(tA + 1), yB0 = ldg(tB), yB1 = ldg(tB + 1);
                float urA = 0.f, urB = 0.f;
                if (qer >= 0.f && ur_check) {
                    urA = ldg(pb.u_right + iA);
                    urB = ldg(pb.u_right + iB);
                }
                auto take = [&](bool ok, float ur, int p, const ulonglong2& y0, const ulonglong2& y1) {
                    if (!ok || (ur > 0 && fabsf(qur - ur) > qer)) return;
                    const int d = __popcll(q0 ^ y0.x) + __popcll(q1 ^ y0.y) + __popcll(q2 ^ y1.x) + __popcll(q3 ^ y1.y);
                    seen++;
                    sorted_insert<KL>(k, ((unsigned)d << 13) | (unsigned)p);
                };
                take(okA, urA, pA, yA0, yA1);
                take(okB, urB, pB, yB0, yB1);
            }
        }
    }
}

__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// LDS scratch of grid_sort: one u32 counter per grid cell + the off-grid bucket
constexpr size_t kGridSortScratch = (size_t)(kNumCells + 1) * 4;

// In-place exclusive scan of a[0..n) (u32) by the workgroup: contiguous segments per
// thread, a DPP wave scan, the wave totals through LDS.  Ends with a barrier.
template <int NT>
__device__ void block_exscan_u32(unsigned* a, int n) {
    __shared__ unsigned s_wsum[NT / 64];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int per = (n + NT - 1) / NT, b = t * per, e = min(n, b + per);
    unsigned sum = 0;
    for (int i = b; i < e; i++) sum += a[i];
    const unsigned incl = wave_inclusive_sum(sum);
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    unsigned run = incl - sum;
    for (int w = 0; w < wave; w++) run += s_wsum[w];
    for (int i = b; i < e; i++) {
        const unsigned v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
}

// The frame's keypoints sorted by (grid cell, index) into skey[0..n): a counting sort
// over the cells (Frame::PosInGrid, Frame.cc:558-567; off-grid keypoints last), then
// each cell's few keys put in index order by one thread.  cnt: kGridSortScratch bytes
// of LDS.  Whole workgroup; ends with a barrier.
template <int NT>
__device__ void grid_sort(const ProjProblem& pb, unsigned* skey, unsigned* cnt) {
    const int tid = threadIdx.x, n = pb.n;
    for (int c = tid; c <= kNumCells; c += NT) cnt[c] = 0u;
    __syncthreads();
    for (int i = tid; i < n; i += NT) {
        const orbx_keypoint kp = ldg(pb.keys + i);
        const int px = (int)roundf((kp.x - pb.min_x) * pb.inv_w);
        const int py = (int)roundf((kp.y - pb.min_y) * pb.inv_h);
        const bool in = !(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows);
        atomicAdd(&cnt[in ? px * kGridRows + py : kNumCells], 1u);
    }
    __syncthreads();
    block_exscan_u32<NT>(cnt, kNumCells + 1);
    for (int i = tid; i < n; i += NT) {
        const orbx_keypoint kp = ldg(pb.keys + i);
        const int px = (int)roundf((kp.x - pb.min_x) * pb.inv_w);
        const int py = (int)roundf((kp.y - pb.min_y) * pb.inv_h);
        const bool in = !(px < 0 || px >= kGridCols || py < 0 || py >= kGridRows);
        const int cell = in ? px * kGridRows + py : kNoCell;
        const unsigned slot = atomicAdd(&cnt[in ? cell : kNumCells], 1u);
        skey[slot] = ((unsigned)cell << 18) | ((unsigned)i << 5) | ((unsigned)kp.octave & 31u);
    }
    __syncthreads();
    // cnt[c] is now the end of cell c; a cell holds a handful of keys
    for (int c = tid; c <= kNumCells; c += NT) {
        const int b = c == 0 ? 0 : (int)cnt[c - 1], e = (int)cnt[c];
        for (int i = b + 1; i < e; i++) {
            const unsigned v = skey[i];
            int j = i - 1;
            while (j >= b && skey[j] > v) {
                skey[j + 1] = skey[j];
                j--;
            }
            skey[j + 1] = v;
        }
    }
    __syncthreads();
}

// ORBX_SPLIT_SXY_GLOBAL=1: the sequence matcher's scoring form keeps the sorted keypoint
// positions in its grid record in global memory (where k_seq_commit reads them) instead
// of LDS -- 8 B per keypoint (40 KB at configs[4]) less LDS held beside the extraction
// lanes.  Measured slower (r05r: configs[4] 106.6-108.5k -> 103.8-104.8k frames/s): the
// scoring's own window reads cost more than the LDS frees.
#ifndef ORBX_SPLIT_SXY_GLOBAL
#define ORBX_SPLIT_SXY_GLOBAL 0
#endif
constexpr bool kSplitSxyGlobal = ORBX_SPLIT_SXY_GLOBAL != 0;

// LDS layout of k_proj_search (byte offsets), shared by the kernel and its launcher.
struct ProjLds {
    size_t skey, colstart, bstart, orun, sxy, sfmp, owner, sang, elist, sdesc, qk, qmp, qang, mlist, mbin, total;
    __host__ __device__ ProjLds(int n, int nq, bool dlds, bool qlds, int noct, bool replay = true, bool xy = true) {
        skey = 0;
        colstart = align16((size_t)n * 4);
        bstart = align16(colstart + (size_t)(kGridCols + 1) * 2);
        orun = align16(bstart + (size_t)bucket_table_len(noct) * 2);
        sxy = align16(orun + (size_t)n * 2);
        sfmp = sxy + (xy ? (size_t)n * 8 : 0);  // !xy: the positions live in global memory
        // the claims and the replay's owner map (neither without the replay: the split
        // scoring keeps a keypoint's initial claim as bit 31 of its sorted key)
        owner = sfmp + (replay ? (size_t)n * 4 : 0);
        // keypoint angles in sorted order (the rotation bins), with the LDS-resident query
        // state only; the lean form reads them from the keypoints after the replay
        sang = owner + (replay ? (size_t)n * 4 : 0);
        size_t o = align16(sang + (qlds ? (size_t)n * 4 : 0));
        elist = o;  // the replay wave's lists (kTopK x 64 entries)
        if (replay) o += (size_t)kTopK * 64 * 4;
        sdesc = o;
        if (dlds) o += (size_t)n * 32;
        qk = o;
        qmp = qk + (size_t)nq * 4 * kTopK;
        qang = qmp + (size_t)nq * 4;
        mlist = qang + (size_t)nq * 4;
        mbin = mlist + (size_t)nq * 4;
        total = qlds ? mbin + (size_t)nq * 4 : o;
        // grid_sort's and build_octave_runs' counters, before the fill
        const size_t scr = octave_runs_scratch(noct) > kGridSortScratch ? octave_runs_scratch(noct) : kGridSortScratch;
        if (total < sxy + scr) total = sxy + scr;
    }
};

// Wave 0's sequential replay (H5) of one problem over the per-query candidate lists qk
// (kTopK entries per query) built by the scoring phase: every query takes the first still
// unclaimed entries of its list (claims only ever block more keypoints, so these are its
// exact best / second best while the list has them), resolved 64 queries at a time as a
// fixpoint (below); a query whose list ran out is re-scored against the current claims;
// then the rotation histogram (ORBmatcher.cc:1750-1786, 1935-1977).  sfmp / owner: the
// claims and the owner map by sorted position (LDS, owner initialised to 0x7fffffff);
// elist: kTopK x 64 words of LDS; angle_of(p): the angle of the keypoint at sorted
// position p.  Whole wave active.  (The previous form committed the chunk's prefix
// before its first conflict per round: configs[4] 447 rounds and 796 us per problem
// against 191 iterations and 445 us for this one, configs[1] 73 -> 59 us.)
template <typename AngleFn>
__device__ void proj_replay(const ProjProblem& pb, const ProjParams& P, const SortedGrid& G, int* sfmp, int* owner,
                            unsigned* elist, const uint4* qk, const int* qmp, const float* qang, int* mlist,
                            int* mbin, int* s_hist, AngleFn angle_of, unsigned long long* st) {
    const int lane = threadIdx.x & 63;
    const int nq = pb.nq;
    int nmatch = 0, nrec = 0, nrescore = 0, niter = 0, ntrunc = 0;
    // diagnostics (stamps): re-scoring, chunk loads + first round, chunk loads alone
    unsigned long long t_res = 0, t_first = 0, t_load = 0;
    const float factor = kHistoLength / 360.0f;
    const int need = P.ratio_mode ? 2 : 1;
    const unsigned long long below = (1ull << lane) - 1;
    // Fixpoint form.  The reference's loop is a function of the query order: query l's
    // choice (first two unclaimed entries, acceptance) depends only on the claims of the
    // queries before it.  Within a 64-query chunk every lane evaluates its choice against
    // the committed claims plus the current proposals of the earlier lanes (an LDS owner
    // map: owner[p] = lowest lane proposing p), and all lanes re-evaluate together until
    // no lane changes (Jacobi iteration: after t iterations the first t lanes are final,
    // so it converges, and its fixpoint is the sequential result).  A chunk with k
    // independent conflicts then costs one iteration plus the longest dependency chain,
    // not k rounds.  A lane whose list ran out stops the commit (it is re-scored against
    // the committed claims); a lane accepting a MapPoint whose claim does not block (a11:
    // Observations() == 0) does not -- later lanes ignore its proposal, and the commit
    // keeps the last claim of a keypoint.
    const int lastp = pb.n > 0 ? pb.n - 1 : 0;
    int guard = 0;
    // a chunk's lists, MapPoints and queries (the latter for a re-scoring) are loaded
    // while the chunk before it replays
    uint4 nx_l[kListVec];
    int nx_mp = -1;
    QueryReg nx_q;
    // Unconditional loads (a clamped index; nx_ok marks the real ones): a load under a
    // per-lane branch makes the compiler merge its registers at the join, which waits for
    // the data at once and turns the prefetch into a stall.
    bool nx_ok = false;
    auto fetch = [&](int qn) {
        const int qc = min(qn, nq - 1);  // nq >= 1 wherever fetch runs
        nx_ok = qn < nq;
        nx_q = load_query(pb, qc);
        nx_mp = qmp[qc];
#pragma unroll
        for (int v = 0; v < kListVec; v++) nx_l[v] = qk[kListVec * qc + v];
    };
    if (nq > 0) fetch(lane);
    for (int base = 0; base < nq && guard >= 0; base += 64) {
        const int q = base + lane;
        const unsigned long long t_chunk = st ? wall_clock64() : 0;
        int mp = nx_ok ? nx_mp : -1;
        unsigned e[kTopK];
#pragma unroll
        for (int v = 0; v < kListVec; v++) {
            e[4 * v] = mp >= 0 ? nx_l[v].x : kNoEntry;
            e[4 * v + 1] = mp >= 0 ? nx_l[v].y : kNoEntry;
            e[4 * v + 2] = mp >= 0 ? nx_l[v].z : kNoEntry;
            e[4 * v + 3] = mp >= 0 ? nx_l[v].w : kNoEntry;
        }
        const QueryReg mine = nx_q;  // consumed only by a re-scoring
        fetch(q + 64);
        // Per lane, derived once per list (at the chunk's start and after a re-scoring):
        // the list itself in LDS (elist[j][lane]: an entry is picked by a per-lane index,
        // conflict-free), its entries' owner-map slots, vm = the real entries (bits), full =
        // it may hide unlisted candidates, lastgt = its last real entry is beyond the
        // acceptance threshold.
        unsigned vm = 0;
        bool full = false, lastgt = false;
        int oa[kTopK];
        auto set_list = [&]() {
            vm = 0;
            int lastd = -1;
#pragma unroll
            for (int j = 0; j < kTopK; j++) {
                elist[j * 64 + lane] = e[j];
                oa[j] = min(ent_pos(e[j]), lastp);
                vm |= (e[j] < kTrunc ? 1u : 0u) << j;
                if (e[j] < kTrunc) lastd = ent_dist(e[j]);
            }
            full = e[kTopK - 1] != kNoEntry;
            lastgt = lastd > P.accept_th;
        };
        set_list();
        // this lane's claims block later queries (a11: only a MapPoint with observations)
        bool bself = false;
        // cblk bit j: entry j is taken by a committed claim (the claims before the chunk:
        // one batch of independent LDS reads, and Observations() loads for a11)
        unsigned cblk = 0;
        if (mp >= 0) {
            bself = claim_blocks(mp);
#pragma unroll
            for (int j = 0; j < kTopK; j++) cblk |= (claim_blocks(sfmp[oa[j]]) ? 1u : 0u) << j;
        }
        // a lane's choice given the blocked entries bm: c1 (its best free entry), whether
        // it accepts c1, and whether its list ran out (exhausted: unlisted candidates may
        // be the answer).  Bit arithmetic on the free mask; c1 / c2 read from elist.
        unsigned c1 = kNoEntry;
        bool exh = false, acc = false;
        auto eval = [&](unsigned bm) {
            const unsigned fm = vm & ~bm;
            const int cnt = __popc(fm);
            const unsigned a1 = fm ? elist[__builtin_ctz(fm) * 64 + lane] : kNoEntry;
            // a full (or truncated) list may hide unlisted candidates -- but they are at
            // least as far as its last exact entry (the list holds the smallest keys), so
            // when that entry, or the free c1 of a ratio test, is already beyond the
            // acceptance threshold the query stays unmatched
            bool x = full && cnt < need;
            if (x && ((cnt == 0 && lastgt) || (cnt == 1 && ent_dist(a1) > P.accept_th))) x = false;
            bool a = !x && fm != 0 && ent_dist(a1) <= P.accept_th;
            if (a && P.ratio_mode) {
                const unsigned f2 = fm & (fm - 1);
                const unsigned a2 = f2 ? elist[__builtin_ctz(f2) * 64 + lane] : kNoEntry;
                const int bestLevel2 = a2 == kNoEntry ? -1 : ent_oct(a2);
                const int bestDist2 = a2 == kNoEntry ? 256 : ent_dist(a2);
                if (ent_oct(a1) == bestLevel2 && (float)ent_dist(a1) > P.nnratio * (float)bestDist2) a = false;
            }
            c1 = a1;
            exh = x;
            acc = a;
        };
        // what later lanes and the commit see of a lane's choice
        auto sig = [&]() { return exh ? kTrunc : (acc ? c1 : kNoEntry); };
        if (mp >= 0) eval(cblk);
        if (st) t_load += wall_clock64() - t_chunk;
        int start = 0;
        int ow[kTopK];
        bool first = true;
        while (true) {
            niter++;
            if (++guard > 66 * (nq + 64)) {  // never reached: <= 65 iterations per fixpoint
                guard = -1;
                break;
            }
            const bool act = lane >= start && mp >= 0;
            const int prop = act && acc && bself ? ent_pos(c1) : -1;
            const unsigned old = sig();
            // owner[p] = lowest lane proposing p (LDS ops of a wave are executed in order:
            // all atomics, then all reads, then the reset)
            if (prop >= 0) atomicMin(&owner[prop], lane);
#pragma unroll
            for (int j = 0; j < kTopK; j++) ow[j] = owner[oa[j]];  // every lane: no exec-masked reads
            if (prop >= 0) owner[prop] = 0x7fffffff;
            // bit j: entry j proposed by an earlier lane (ow - lane < 0; ow >= 0, lane < 64)
            unsigned sb = 0;
#pragma unroll
            for (int j = 0; j < kTopK; j++) sb |= ((unsigned)(ow[j] - lane) >> 31) << j;
            if (act) eval(cblk | sb);
            if (__ballot(act && sig() != old)) continue;
            // fixpoint: every active lane's choice is the sequential one up to the first
            // exhausted lane f
            const unsigned long long sm = __ballot(act && exh);
            const int f = sm ? __ffsll((long long)sm) - 1 : 64;
            const bool com = act && acc && lane < f;
            const unsigned long long comm = __ballot(com);
            // Blocking claims are unique (a later lane saw them).  A non-blocking claim
            // (a11: Observations() == 0) may be taken again by a later lane of the same
            // commit, which then keeps the keypoint (ORBmatcher.cc:117-119, 167): it is
            // written only by the last lane claiming its keypoint (owner map: the lowest
            // 63 - lane, in order: atomics, reads, reset).
            if (com && bself) sfmp[ent_pos(c1)] = mp;
            if (__ballot(com && !bself)) {
                const int pp = com ? ent_pos(c1) : 0;
                if (com) atomicMin(&owner[pp], 63 - lane);
                const int lo = owner[pp];
                if (com) owner[pp] = 0x7fffffff;
                if (com && !bself && lo == 63 - lane) sfmp[pp] = mp;
            }
            nmatch += __popcll(comm);
            if (P.check_ori) {
                // the match is recorded with its query; the rotation bins are computed
                // after the replay, off the sequential path
                if (com) {
                    const int r = nrec + __popcll(comm & below);
                    mlist[r] = ent_pos(c1);
                    mbin[r] = q;
                }
                nrec += __popcll(comm);
            }
            if (st && first) t_first += wall_clock64() - t_chunk;
            first = false;
            if (f >= 64) break;
            // the committed lanes' claims, for the lanes after them: the entries a lane
            // below f proposed (blocking proposals only reach the owner map)
#pragma unroll
            for (int j = 0; j < kTopK; j++) cblk |= (act && lane >= f ? (unsigned)(ow[j] - f) >> 31 : 0u) << j;
            start = f;
            {
                // lane f's list ran out: re-score it against the current claims.  Any list
                // that is exact against the claims of some moment stays valid later
                // (claims only ever block more keypoints), so the other exhausted lanes
                // of the chunk are re-scored in the same pass, one 16-lane row each.
                const unsigned long long t0 = st ? wall_clock64() : 0;
                wave_lds_fence();
                unsigned long long X = __ballot(act && exh && lane >= f);
                if (st) {  // diagnostics: the list ran out at a truncation, not at its last entry
                    bool tr = false;
#pragma unroll
                    for (int j = 0; j < kTopK; j++) tr = tr || e[j] == kTrunc;
                    ntrunc += __builtin_amdgcn_readlane((int)tr, f);
                }
                unsigned ne[kTopK];
                if (__popcll(X) > 1) {
                    // rows 0..3 take the first four exhausted lanes
                    const int row = lane >> 4;
                    unsigned long long x = X;
                    for (int r = 0; r < row; r++) x &= x - 1;
                    const bool valid = x != 0;
                    const int src = valid ? __ffsll((long long)x) - 1 : f;
                    score_groupk<16>(pb, P, shfl_query(mine, src), valid, G, sfmp, ne);
                    const int myrow = __popcll(X & below);
                    const bool mine_row = ((X >> lane) & 1ull) && myrow < 4;
#pragma unroll
                    for (int j = 0; j < kTopK; j++) {
                        const unsigned v = (unsigned)__shfl((int)ne[j], (myrow & 3) * 16);
                        if (mine_row) e[j] = v;
                    }
                    nrescore += __popcll(X) < 4 ? __popcll(X) : 4;
                    if (mine_row) {
                        cblk = 0;
                        set_list();
                        eval(0);
                    }
                } else {
                    score_groupk<64>(pb, P, bcast_query(mine, f), true, G, sfmp, ne);  // wave-uniform result
#pragma unroll
                    for (int j = 0; j < kTopK; j++)
                        if (lane == f) e[j] = ne[j];
                    nrescore++;
                    if (lane == f) {
                        cblk = 0;  // the new list holds free keypoints only
                        set_list();
                        eval(0);   // lane f is the first active lane: no earlier proposals
                    }
                }
                if (st) t_res += wall_clock64() - t0;
            }
            wave_lds_fence();
        }
        wave_lds_fence();
    }
    if (st && lane == 0) st[15] = wall_clock64();
    if (guard < 0) nmatch = -1;  // a broken fixpoint (never observed): fail the parity check loudly
    // the match list (global scratch in some modes) is read back by other lanes below
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    if (P.check_ori) {
        // rotHist of the committed matches (ORBmatcher.cc:1750-1757): bin of (query angle
        // - keypoint angle); integer counts, so the order of the additions is immaterial
        for (int m = lane; m < nrec; m += 64) {
            const int tpos = mlist[m];
            float rot = qang[mbin[m]] - angle_of(tpos);
            if (rot < 0.0f) rot += 360.0f;
            int bin = (int)roundf(rot * factor);
            if (bin == kHistoLength) bin = 0;
            mbin[m] = bin;
            atomicAdd(&s_hist[bin], 1);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    if (P.check_ori) {
        // ComputeThreeMaxima, ORBmatcher.cc:1935-1977
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < kHistoLength; i++) {
            const int s = s_hist[i];
            if (s > max1) {
                max3 = max2; max2 = max1; max1 = s;
                ind3 = ind2; ind2 = ind1; ind1 = i;
            } else if (s > max2) {
                max3 = max2; max2 = s;
                ind3 = ind2; ind2 = i;
            } else if (s > max3) {
                max3 = s;
                ind3 = i;
            }
        }
        if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
        int bad = 0;
        for (int m = lane; m < nrec; m += 64) {
            const int b = mbin[m];
            if (b != ind1 && b != ind2 && b != ind3) {
                sfmp[mlist[m]] = -1;
                bad++;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o);
        nmatch -= bad;
    }
    if (lane == 0) *pb.nmatches = nmatch;
    if (st && lane == 0) {
        st[3] = wall_clock64();
        st[5] = nrescore;
        st[12] = ntrunc;
        st[6] = nq;
        st[7] = niter;
        st[8] = t_res;
        st[9] = t_first;
        st[14] = t_load;
        st[kStampForm] = 64;
    }
}

// The replay over RT threads (RT / 64 waves): the fixpoint of proj_replay over chunks of
// RT queries instead of 64.  The iterations a chunk takes are set by its longest
// dependency chain, not by its size, so wider chunks mean fewer iterations per query;
// every exhausted list of a chunk is re-scored at the first sequence point (each wave
// its own lanes, four per 16-lane-row pass), so a chunk rarely stops twice.
// owner[p] (zero-initialised, n words): (iteration << 10 | 1023 - thread) of the lowest
// thread proposing p this iteration (atomicMax; stale iterations are ignored, so the map
// is never reset).  elist: kTopK x RT words.  Whole workgroup of RT threads.
template <int RT, typename AngleFn>
__device__ void proj_replay_block(const ProjProblem& pb, const ProjParams& P, const SortedGrid& G, int* sfmp,
                                  unsigned* owner, unsigned* elist, const uint4* qk, const int* qmp,
                                  const float* qang, int* mlist, int* mbin, int* s_hist, AngleFn angle_of,
                                  unsigned long long* st) {
    static_assert(RT % 64 == 0 && RT <= 1024, "whole waves, 10-bit thread tags");
    constexpr int kW = RT / 64;
    __shared__ int s_key;
    __shared__ int s_wc[kW];
    __shared__ int s_bad;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nq = pb.nq;
    const int lastp = pb.n > 0 ? pb.n - 1 : 0;
    const int need = P.ratio_mode ? 2 : 1;
    const unsigned long long below = (1ull << lane) - 1;
    const float factor = kHistoLength / 360.0f;
    int nmatch = 0, nrec = 0, nrescore = 0, niter = 0, nstop = 0;  // block-uniform
    // diagnostics (stamps, thread 0's clock): chunk loads, fixpoint rounds, commits, re-scoring
    unsigned long long t_load = 0, t_round = 0, t_commit = 0, t_res = 0, tc = 0;
    const bool clk = st && tid == 0;
    unsigned it = 0;
    long long guard = 0;
    bool broken = false;
    if (tid == 0) s_key = 0x7fffffff;
    // a chunk's lists, MapPoints and queries are loaded while the chunk before it replays
    uint4 nx_l[kListVec];
    int nx_mp = -1;
    QueryReg nx_q;
    // Unconditional loads (a clamped index; nx_ok marks the real ones): a load under a
    // per-lane branch makes the compiler merge its registers at the join, which waits for
    // the data at once and turns the prefetch into a stall.
    bool nx_ok = false;
    auto fetch = [&](int qn) {
        const int qc = min(qn, nq - 1);  // nq >= 1 wherever fetch runs
        nx_ok = qn < nq;
        nx_q = load_query(pb, qc);
        nx_mp = qmp[qc];
#pragma unroll
        for (int v = 0; v < kListVec; v++) nx_l[v] = qk[kListVec * qc + v];
    };
    if (nq > 0) fetch(tid);
    __syncthreads();
    for (int base = 0; base < nq && !broken; base += RT) {
        if (it > (1u << 20)) {  // keep iteration << 10 in 31 bits: restart the tags
            for (int p = tid; p < pb.n; p += RT) owner[p] = 0u;
            it = 0;
            __syncthreads();
        }
        const int q = base + tid;
        if (clk) tc = wall_clock64();
        const int mp = nx_ok ? nx_mp : -1;
        unsigned e[kTopK];
#pragma unroll
        for (int v = 0; v < kListVec; v++) {
            e[4 * v] = mp >= 0 ? nx_l[v].x : kNoEntry;
            e[4 * v + 1] = mp >= 0 ? nx_l[v].y : kNoEntry;
            e[4 * v + 2] = mp >= 0 ? nx_l[v].z : kNoEntry;
            e[4 * v + 3] = mp >= 0 ? nx_l[v].w : kNoEntry;
        }
        const QueryReg mine = nx_q;
        fetch(q + RT);
        unsigned vm = 0;
        bool full = false, lastgt = false;
        int oa[kTopK];
        auto set_list = [&]() {
            vm = 0;
            int lastd = -1;
#pragma unroll
            for (int j = 0; j < kTopK; j++) {
                elist[j * RT + tid] = e[j];
                oa[j] = min(ent_pos(e[j]), lastp);
                vm |= (e[j] < kTrunc ? 1u : 0u) << j;
                if (e[j] < kTrunc) lastd = ent_dist(e[j]);
            }
            full = e[kTopK - 1] != kNoEntry;
            lastgt = lastd > P.accept_th;
        };
        set_list();
        bool bself = false;
        unsigned cblk = 0;
        if (mp >= 0) {
            bself = claim_blocks(mp);
#pragma unroll
            for (int j = 0; j < kTopK; j++) cblk |= (claim_blocks(sfmp[oa[j]]) ? 1u : 0u) << j;
        }
        unsigned c1 = kNoEntry;
        bool exh = false, acc = false;
        auto eval = [&](unsigned bm) {
            const unsigned fm = vm & ~bm;
            const int cnt = __popc(fm);
            const unsigned a1 = fm ? elist[__builtin_ctz(fm) * RT + tid] : kNoEntry;
            bool x = full && cnt < need;
            if (x && ((cnt == 0 && lastgt) || (cnt == 1 && ent_dist(a1) > P.accept_th))) x = false;
            bool a = !x && fm != 0 && ent_dist(a1) <= P.accept_th;
            if (a && P.ratio_mode) {
                const unsigned f2 = fm & (fm - 1);
                const unsigned a2 = f2 ? elist[__builtin_ctz(f2) * RT + tid] : kNoEntry;
                const int bestLevel2 = a2 == kNoEntry ? -1 : ent_oct(a2);
                const int bestDist2 = a2 == kNoEntry ? 256 : ent_dist(a2);
                if (ent_oct(a1) == bestLevel2 && (float)ent_dist(a1) > P.nnratio * (float)bestDist2) a = false;
            }
            c1 = a1;
            exh = x;
            acc = a;
        };
        auto sig = [&]() { return exh ? kTrunc : (acc ? c1 : kNoEntry); };
        if (mp >= 0) eval(cblk);
        if (clk) {
            const unsigned long long t = wall_clock64();
            t_load += t - tc;
            tc = t;
        }
        int start = 0;
        unsigned ow[kTopK];
        while (true) {
            niter++;
            if (++guard > 66ll * (nq + RT)) {  // never reached: <= RT + 1 iterations per fixpoint
                broken = true;
                break;
            }
            it++;
            const bool act = tid >= start && mp >= 0;
            const unsigned old = sig();
            if (act && acc && bself) atomicMax(&owner[ent_pos(c1)], (it << 10) | (unsigned)(1023 - tid));
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kTopK; j++) ow[j] = owner[oa[j]];
            // bit j: entry j proposed this iteration by a thread before this one
            unsigned sb = 0;
#pragma unroll
            for (int j = 0; j < kTopK; j++)
                sb |= ((ow[j] >> 10) == it && (int)(1023u - (ow[j] & 1023u)) < tid ? 1u : 0u) << j;
            if (act) eval(cblk | sb);
            if (__syncthreads_or(act && sig() != old)) continue;
            if (clk) {
                const unsigned long long t = wall_clock64();
                t_round += t - tc;
                tc = t;
            }
            // fixpoint: the first exhausted thread f stops the commit (a non-blocking
            // acceptor does not: see proj_replay)
            int key = act && exh ? tid : 0x7fffffff;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) key = min(key, __shfl_xor(key, o));
            if (lane == 0 && key != 0x7fffffff) atomicMin(&s_key, key);
            __syncthreads();
            const int K = s_key;
            const int f = K == 0x7fffffff ? RT : K;
            const bool com = act && acc && tid < f;
            if (com && bself) sfmp[ent_pos(c1)] = mp;  // unique
            const unsigned long long cm = __ballot(com);
            const bool wnb = __ballot(com && !bself) != 0;
            if (lane == 0) s_wc[wave] = __popcll(cm) | (wnb ? 1 << 16 : 0);
            __syncthreads();
            if (tid == 0) s_key = 0x7fffffff;  // read by every thread before the barrier above
            int tot = 0, woff = 0, nb = 0;
#pragma unroll
            for (int w = 0; w < kW; w++) {
                const int c = s_wc[w] & 0xffff;
                nb |= s_wc[w] >> 16;
                woff += w < wave ? c : 0;
                tot += c;
            }
            const unsigned itf = it;
            if (nb) {
                // non-blocking claims: only the last committed thread claiming a keypoint
                // writes it (a fresh tag iteration, highest thread wins)
                it++;
                const unsigned tag = (it << 10) | (unsigned)tid;
                if (com) atomicMax(&owner[ent_pos(c1)], tag);
                __syncthreads();
                if (com && !bself && owner[ent_pos(c1)] == tag) sfmp[ent_pos(c1)] = mp;
                __syncthreads();  // publishes sfmp for the re-scoring and the next chunk
            }
            if (P.check_ori && com) {
                const int r = nrec + woff + __popcll(cm & below);
                mlist[r] = ent_pos(c1);
                mbin[r] = q;
            }
            nmatch += tot;
            if (P.check_ori) nrec += tot;
            if (clk) {
                const unsigned long long t = wall_clock64();
                t_commit += t - tc;
                tc = t;
            }
            if (f >= RT) break;
            nstop++;
            // the committed threads' claims, for the threads after them
            if (act && tid >= f) {
#pragma unroll
                for (int j = 0; j < kTopK; j++)
                    cblk |= ((ow[j] >> 10) == itf && (int)(1023u - (ow[j] & 1023u)) < f ? 1u : 0u) << j;
            }
            start = f;
            {
                // every exhausted list at or after f, against the current claims (sfmp is
                // published by the barrier above)
                unsigned long long X = __ballot(act && exh && tid >= f);
                while (X) {
                    unsigned ne[kTopK];
                    if (__popcll(X) == 1) {
                        const int src = __ffsll((long long)X) - 1;
                        score_groupk<64>(pb, P, bcast_query(mine, src), true, G, sfmp, ne);
#pragma unroll
                        for (int j = 0; j < kTopK; j++)
                            if (lane == src) e[j] = ne[j];
                        nrescore++;
                        if (lane == src) {
                            cblk = 0;
                            set_list();
                            eval(0);
                        }
                        X = 0;
                    } else {
                        const int row = lane >> 4;
                        unsigned long long x = X;
                        for (int r = 0; r < row; r++) x &= x - 1;
                        const bool valid = x != 0;
                        const int src = valid ? __ffsll((long long)x) - 1 : 0;
                        score_groupk<16>(pb, P, shfl_query(mine, src), valid, G, sfmp, ne);
                        const int myrow = __popcll(X & below);
                        const bool take = ((X >> lane) & 1ull) && myrow < 4;
#pragma unroll
                        for (int j = 0; j < kTopK; j++) {
                            const unsigned v = (unsigned)__shfl((int)ne[j], (myrow & 3) * 16);
                            if (take) e[j] = v;
                        }
                        nrescore += __popcll(X) < 4 ? __popcll(X) : 4;
                        if (take) {
                            cblk = 0;
                            set_list();
                            eval(0);
                        }
                        for (int r = 0; r < 4 && X; r++) X &= X - 1;
                    }
                }
            }
            if (st) __syncthreads();  // diagnostics: every wave's re-scoring done before the clock
            if (clk) {
                const unsigned long long t = wall_clock64();
                t_res += t - tc;
                tc = t;
            }
        }
        __syncthreads();
    }
    // every thread keeps the same counters; the match list is complete after the barrier
    __syncthreads();
    if (P.check_ori && !broken) {
        // rotHist of the committed matches (ORBmatcher.cc:1750-1757)
        for (int m = tid; m < nrec; m += RT) {
            const int tpos = mlist[m];
            float rot = qang[mbin[m]] - angle_of(tpos);
            if (rot < 0.0f) rot += 360.0f;
            int bin = (int)roundf(rot * factor);
            if (bin == kHistoLength) bin = 0;
            mbin[m] = bin;
            atomicAdd(&s_hist[bin], 1);
        }
        if (tid == 0) s_bad = 0;
        __syncthreads();
        // ComputeThreeMaxima, ORBmatcher.cc:1935-1977 (every thread, same result)
        int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
        for (int i = 0; i < kHistoLength; i++) {
            const int s = s_hist[i];
            if (s > max1) {
                max3 = max2; max2 = max1; max1 = s;
                ind3 = ind2; ind2 = ind1; ind1 = i;
            } else if (s > max2) {
                max3 = max2; max2 = s;
                ind3 = ind2; ind2 = i;
            } else if (s > max3) {
                max3 = s;
                ind3 = i;
            }
        }
        if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
        else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
        int bad = 0;
        for (int m = tid; m < nrec; m += RT) {
            const int b = mbin[m];
            if (b != ind1 && b != ind2 && b != ind3) {
                sfmp[mlist[m]] = -1;
                bad++;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o);
        if (lane == 0 && bad) atomicAdd(&s_bad, bad);
        __syncthreads();
        nmatch -= s_bad;
    }
    if (tid == 0) *pb.nmatches = broken ? -1 : nmatch;  // a broken fixpoint (never observed) fails parity loudly
    if (st && tid == 0) {
        st[3] = wall_clock64();
        st[5] = nrescore;
        st[6] = nq;
        st[7] = niter;
        st[8] = t_res;
        st[9] = t_round;
        st[12] = nstop;
        st[14] = t_load;
        st[15] = t_commit;
        st[kStampForm] = RT;
    }
    __syncthreads();
}

// Byte layout of one problem's grid in the global grid area.
struct SeqGridLayout {
    size_t skey, bstart, orun, sxy, sang, sfmp, sdesc, total;
    __host__ __device__ SeqGridLayout(int cap, int noct) {
        skey = 0;
        bstart = align16((size_t)cap * 4);
        orun = align16(bstart + (size_t)bucket_table_len(noct) * 2);
        sxy = align16(orun + (size_t)cap * 2);
        sang = align16(sxy + (size_t)cap * 8);
        sfmp = align16(sang + (size_t)cap * 4);  // the claims (mvpMapPoints) before the search, sorted
        sdesc = align16(sfmp + (size_t)cap * 4);
        total = (sdesc + (size_t)cap * 32 + 255) & ~(size_t)255;
    }
};

__device__ __forceinline__ SortedGrid seq_grid(unsigned char* base, const SeqGridLayout& g, int noct) {
    return SortedGrid{(const unsigned*)(base + g.skey), (const uint16_t*)(base + g.bstart),
                      (const uint16_t*)(base + g.orun), (const float2*)(base + g.sxy),
                      (const uint4*)(base + g.sdesc), noct};
}

// One workgroup per problem (one SearchByProjection call).
//  1. the frame's keypoints are sorted into grid order in LDS (with their descriptors
//     when DLDS);
//  2. all waves score the queries against the initial mvpMapPoints state, keeping each
//     query's four best candidates;
//  3. wave 0 replays the reference's sequential loop 64 queries at a time: every query
//     takes the first candidates of its list that are still unclaimed; the queries of
//     a chunk whose choice no earlier query of the chunk touches commit together, the
//     first one that is touched resumes the replay after the others have committed, and
//     a query whose list ran out is re-scored against the current claims;
//  4. the rotation histogram (ORBmatcher.cc:1750-1786) un-matches bins outside the
//     three maxima.
// Claims only ever block more keypoints during the replay (a blocked keypoint is never
// claimed again), so the first unblocked entries of a query's initial list are exactly
// its best / second best against the current state while the list has them.
// QLDS: per-query state in LDS; otherwise in the problem's global scratch.
// SPLIT: no replay here -- the sorted grid is published to `grids` (SeqGridLayout, no
// sorted descriptors) and k_seq_commit replays with one wave and a small LDS footprint.
// Register budgets (waves per SIMD) of the batched sequence matcher's two kernels, which run
// beside the extraction lanes: every VGPR they hold for their whole launch is one the
// extraction's waves on that SIMD cannot have.  0: the compiler's choice (100 VGPRs for
// the scoring kernel).  The scoring kernel at 5 (96 VGPRs, 20 B of spill) measured +1-2 %
// at configs[4] before the octree split (r05p) and within noise after it (r05af); 6 and 8
// (more spills) and the commit at 3 or 4 measured slower (r05p).
#ifndef ORBX_SCORE_WPE
#define ORBX_SCORE_WPE 0
#endif
#ifndef ORBX_COMMIT_WPE
#define ORBX_COMMIT_WPE 0
#endif
#if ORBX_SCORE_WPE
#define ORBX_SCORE_ATTR __attribute__((amdgpu_waves_per_eu(ORBX_SCORE_WPE)))
#else
#define ORBX_SCORE_ATTR
#endif
#if ORBX_COMMIT_WPE
#define ORBX_COMMIT_ATTR __attribute__((amdgpu_waves_per_eu(ORBX_COMMIT_WPE)))
#else
#define ORBX_COMMIT_ATTR
#endif

template <bool QLDS, bool DLDS, int NT, bool SPLIT>
__device__ __forceinline__ void proj_search_body(const ProjProblem* __restrict__ probs, ProjParams P,
                                                 unsigned long long* __restrict__ scratch,
                                                 const long long* __restrict__ scratch_off,
                                                 unsigned char* __restrict__ grids, int gcap) {
    static_assert(!SPLIT || !DLDS, "the split scoring tests the initial claims through the sorted keys only");
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_hist[kHistoLength];
    const ProjProblem pb = probs[blockIdx.x];
    if (pb.nq < 0) return;  // a pair the retry pass skips (k_seq_build): whole workgroup
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kWaves = NT / 64;
    const int n = pb.n, nq = pb.nq;
    unsigned long long* st = P.stamps ? P.stamps + kStampWords * blockIdx.x : nullptr;
    if (st && tid == 0) st[0] = wall_clock64();
    constexpr bool kXyGlobal = SPLIT && kSplitSxyGlobal;
    const ProjLds L(n, nq, DLDS, QLDS, P.noct, !SPLIT, !kXyGlobal);
    unsigned* skey = (unsigned*)(smem + L.skey);
    uint16_t* colstart = (uint16_t*)(smem + L.colstart);
    uint16_t* bstart = (uint16_t*)(smem + L.bstart);
    uint16_t* orun = (uint16_t*)(smem + L.orun);
    float2* sxy;
    if constexpr (kXyGlobal) {
        const SeqGridLayout gl(gcap, P.noct);
        sxy = (float2*)(grids + (size_t)blockIdx.x * gl.total + gl.sxy);
    } else {
        sxy = (float2*)(smem + L.sxy);
    }
    int* sfmp = (int*)(smem + L.sfmp);
    int* owner = (int*)(smem + L.owner);
    float* sang = (float*)(smem + L.sang);
    uint4* sdesc = DLDS ? (uint4*)(smem + L.sdesc) : nullptr;
    uint4* qk;
    int *qmp, *mlist, *mbin;
    float* qang;
    if (QLDS) {
        qk = (uint4*)(smem + L.qk);
        qmp = (int*)(smem + L.qmp);
        qang = (float*)(smem + L.qang);
        mlist = (int*)(smem + L.mlist);
        mbin = (int*)(smem + L.mbin);
    } else {
        unsigned long long* g = scratch + scratch_off[blockIdx.x];
        qk = (uint4*)g;
        qmp = (int*)(g + kListWords * (size_t)nq);
        qang = (float*)(qmp + nq);
        mlist = (int*)(qang + nq);
        mbin = mlist + nq;
    }
    if (tid < kHistoLength) s_hist[tid] = 0;
    grid_sort<NT>(pb, skey, (unsigned*)(smem + L.sxy));  // counters where the keypoint state goes next
    if (st && tid == 0) st[10] = wall_clock64();
    build_colstart<NT>(skey, n, colstart);
    __syncthreads();
    if (st && tid == 0) st[11] = wall_clock64();
    // the octave runs' counters live where the per-keypoint state goes next
    build_octave_runs<NT>(skey, colstart, P.noct, bstart, orun, (unsigned*)(smem + L.sxy));
    __syncthreads();
    for (int p = tid; p < n; p += NT) {
        const unsigned k = skey[p];
        const int i = sk_idx(k);
        const orbx_keypoint kp = ldg(pb.keys + i);
        sxy[p] = make_float2(kp.x, kp.y);
        if (SPLIT) {
            if (kp_blocked(ldg(pb.frame_mp + i), P)) skey[p] = k | kKeyBlocked;
        } else {
            sfmp[p] = claim_word(ldg(pb.frame_mp + i), P);
            owner[p] = 0x7fffffff;
        }
        if (QLDS) sang[p] = kp.angle;
    }
    if (DLDS) {
        for (int t = tid; t < 2 * n; t += NT) {
            const int i = sk_idx(skey[t >> 1]);
            sdesc[t] = ldg((const uint4*)(pb.desc + (size_t)i * 32) + (t & 1));
        }
    }
    __syncthreads();
    if (st && tid == 0) st[1] = wall_clock64();
    const SortedGrid G{skey, bstart, orun, sxy, sdesc, P.noct};
    // KR lanes per query, by the width of the query's cell window: a row's lanes split the
    // window's columns, and its merge (kTopK rounds of a KR-lane minimum) costs the same
    // however few candidates the window holds.  Until round 4 one KR for all queries (8 up
    // to 8 pyramid levels, 16 above); now the queries are cut into three index ranges by a
    // count of their window widths -- KR 4 for at most ~4 columns, 8 for ~8, 16 beyond --
    // which are the exact classes when the queries come in octave order (TrackWithMotion-
    // Model's LastFrame keypoints are level-major) and otherwise only a cost heuristic: the
    // lists do not depend on KR.  ORBX_SCORE_KR_FIXED=1 builds the round-4 choice.
    __shared__ int s_qcut[2];
    // Pyramids of up to 8 levels keep KR 8 for every query: the classes measured slower
    // there (configs[1] 227.8-228.4k -> 224.3-225.9k frames/s) and faster above
    // (configs[4] 108.2-108.3k -> 111.1-111.3k; r05c, interleaved on one box).
    // The split scoring (the sequence matcher beside the extraction) gives every query the
    // same kSplitKr lanes instead.
    const bool one_kr = ORBX_SCORE_KR_FIXED || P.noct <= 8 || (SPLIT && kSplitKr > 0);  // uniform over the workgroup
    __shared__ int s_next;  // score_pairs' query counter
    if (tid < 2) s_qcut[tid] = one_kr && tid == 1 && P.noct <= 8 ? nq : 0;
    if (tid == 0) s_next = 0;
    __syncthreads();
    if (!one_kr) {
        int c4 = 0, c8 = 0;
        for (int q = tid; q < nq; q += NT) {
            const float w = 2.0f * ldg(&pb.q[q].r) * pb.inv_w;  // window width in cells
            c4 += w <= 2.0f;
            c8 += w <= 6.0f;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            c4 += __shfl_xor(c4, o);
            c8 += __shfl_xor(c8, o);
        }
        if (lane == 0 && (c4 | c8)) {
            atomicAdd(&s_qcut[0], c4);
            atomicAdd(&s_qcut[1], c8);
        }
    }
    __syncthreads();
    const int qcut4 = s_qcut[0], qcut8 = s_qcut[1];
    constexpr bool kPrefetch = !SPLIT || ORBX_SPLIT_PREFETCH;  // the next queries' loads during the current ones
    auto pass = [&](auto kr, int q0, int q1) {
        constexpr int KR = decltype(kr)::value;
        constexpr int kQw = 64 / KR;  // queries per wave and pass
        constexpr int kStep = kWaves * kQw;
        int qb = q0 + wave * kQw;
        QueryReg cur;
        if (qb < q1) cur = load_query(pb, min(qb + lane / KR, q1 - 1));
        for (; qb < q1; qb += kStep) {
            const int q = qb + lane / KR;
            QueryReg nxt;
            if (kPrefetch && qb + kStep < q1) nxt = load_query(pb, min(q + kStep, q1 - 1));  // prefetch
            const int mp = q < q1 ? cur.q.mp : -1;
            unsigned e[kTopK];
            score_groupk<KR, SPLIT ? split_lane_topk(KR) : kLaneTopK>(pb, P, cur, mp >= 0, G, SPLIT ? nullptr : sfmp, e);
            if ((lane & (KR - 1)) == 0 && q < q1) {
#pragma unroll
                for (int v = 0; v < kListVec; v++)
                    qk[kListVec * q + v] = make_uint4(e[4 * v], e[4 * v + 1], e[4 * v + 2], e[4 * v + 3]);
                qmp[q] = claim_word(mp, P);
                qang[q] = cur.q.angle;
            }
            if (kPrefetch)
                cur = nxt;
            else if (qb + kStep < q1)
                cur = load_query(pb, min(q + kStep, q1 - 1));
        }
    };
    if constexpr (SPLIT && kSplitKr > 0) {
        // pyramids above eight levels: the pairs without lockstep (configs[4] RGB-D +2.2 %; at
        // configs[1] they measured 1 % slower than the lockstep pairs, r06pq)
        if (ORBX_SPLIT_PERSIST && P.noct > 8)
            score_pairs(pb, P, G, qk, qmp, qang, &s_next);
        else
            pass(std::integral_constant<int, (kSplitKr > 0 ? kSplitKr : 1)>{}, 0, nq);
    } else {
        if (qcut4 > 0) pass(std::integral_constant<int, 4>{}, 0, qcut4);
        if (qcut8 > qcut4) pass(std::integral_constant<int, 8>{}, qcut4, qcut8);
        if (nq > qcut8) pass(std::integral_constant<int, 16>{}, qcut8, nq);
    }
    __syncthreads();
    if (st && tid == 0) st[2] = wall_clock64();
    if (SPLIT) {
        const SeqGridLayout gl(gcap, P.noct);
        unsigned char* gb = grids + (size_t)blockIdx.x * gl.total;
        const int nb = bucket_table_len(P.noct);
        for (int p = tid; p < n; p += NT) {
            ((unsigned*)(gb + gl.skey))[p] = skey[p] & ~kKeyBlocked;
            ((uint16_t*)(gb + gl.orun))[p] = orun[p];
            if (!kXyGlobal) ((float2*)(gb + gl.sxy))[p] = sxy[p];
            ((float*)(gb + gl.sang))[p] = ldg(&pb.keys[sk_idx(skey[p])].angle);
        }
        for (int t = tid; t < nb; t += NT) ((uint16_t*)(gb + gl.bstart))[t] = bstart[t];
        return;
    }
    // The replay is wave 0's alone: the other waves leave now, so their registers and
    // wave slots go back to whatever runs beside this kernel for the rest of its life.
    if (wave != 0) return;
    proj_replay(pb, P, G, sfmp, owner, (unsigned*)(smem + L.elist), qk, qmp, qang, mlist, mbin, s_hist,
                [&](int tpos) { return QLDS ? sang[tpos] : ldg(&pb.keys[sk_idx(skey[tpos])].angle); }, st);
    wave_lds_fence();
    for (int p = lane; p < n; p += 64) pb.frame_mp[sk_idx(skey[p])] = claim_mp(sfmp[p]);
    if (st && lane == 0) st[4] = wall_clock64();
}

template <bool QLDS, bool DLDS, int NT, bool SPLIT = false>
__global__ __launch_bounds__(NT) void k_proj_search(const ProjProblem* __restrict__ probs, ProjParams P,
                                                    unsigned long long* __restrict__ scratch,
                                                    const long long* __restrict__ scratch_off,
                                                    unsigned char* __restrict__ grids, int gcap) {
    proj_search_body<QLDS, DLDS, NT, SPLIT>(probs, P, scratch, scratch_off, grids, gcap);
}

// the sequence matcher's scoring form (beside the extraction lanes) with its register budget
template <>
__global__ __launch_bounds__(kSplitScoreThreads) ORBX_SCORE_ATTR void k_proj_search<false, false, kSplitScoreThreads, true>(
    const ProjProblem* __restrict__ probs, ProjParams P, unsigned long long* __restrict__ scratch,
    const long long* __restrict__ scratch_off, unsigned char* __restrict__ grids, int gcap) {
    proj_search_body<false, false, kSplitScoreThreads, true>(probs, P, scratch, scratch_off, grids, gcap);
}

// ---- the batched sequence matcher in three launches (orbx_match_sequence_device)
//
// k_proj_search keeps a whole workgroup per problem for the grid sort, the scoring and
// the replay, so most of its lifetime is one wave replaying while the rest of the
// workgroup's slots and LDS sit idle beside the extraction.  The sequence path splits it:
//   k_seq_grid    one workgroup per problem: the current frame's keypoints sorted into
//                 grid order (the SortedGrid, here in global memory, with the sorted
//                 descriptors and angles);
//   k_seq_score   16 queries per workgroup over all problems (XCD-aware: a problem's
//                 workgroups share one L2 with its grid): each query's kTopK-entry list;
//   k_seq_commit  one wave per problem: the replay (proj_replay) with the claims in LDS.
// Results are identical to k_proj_search's (same lists, same replay).

constexpr int kSeqGridThreads = 256;

hipError_t launch_stage_copy(const void* src, void* dst, size_t bytes, hipStream_t stream);

// A single host call's inputs, copied from device-visible pinned host memory into the
// device arena by the GPU itself (many workgroups of coalesced 16-byte loads over PCIe)
// rather than by a DMA copy: the copy engine's setup latency is most of a small copy's
// cost, and one workgroup alone reads host memory at only ~7 GB/s (21 us for 150 KB).
constexpr int kStageThreads = 256, kStageUnroll = 4;
__global__ __launch_bounds__(kStageThreads) void k_stage_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                              int n16) {
    const int b0 = blockIdx.x * kStageThreads * kStageUnroll + (int)threadIdx.x;
    uint4 v[kStageUnroll];
#pragma unroll
    for (int u = 0; u < kStageUnroll; u++) {
        const int i = b0 + u * kStageThreads;
        if (i < n16) v[u] = src[i];
    }
#pragma unroll
    for (int u = 0; u < kStageUnroll; u++) {
        const int i = b0 + u * kStageThreads;
        if (i < n16) dst[i] = v[u];
    }
}

template <int kSeqGridThreads>  // (shadows the batch default of the same name)
__global__ __launch_bounds__(kSeqGridThreads) void k_seq_grid(const ProjProblem* probs, ProjParams P, unsigned char* grids,
                                                              int cap, int noct, unsigned long long* stamps) {
    extern __shared__ __align__(16) unsigned char smem[];
    // diagnostics (one problem): words 0, 1, 2, 4, 10, 11 of its stamp row
    unsigned long long* st = stamps && threadIdx.x == 0 ? stamps + kStampWords * blockIdx.x : nullptr;
    if (st) st[0] = wall_clock64();
    if (st) st[1] = wall_clock64();
    const ProjProblem pb = probs[blockIdx.x];
    if (pb.nq < 0) return;  // skipped by the retry pass
    const SeqGridLayout gl(cap, noct);
    unsigned char* gb = grids + (size_t)blockIdx.x * gl.total;
    const int tid = threadIdx.x, n = pb.n;
    // LDS: skey [cap], colstart [kGridCols + 1], counters
    unsigned* skey = (unsigned*)smem;
    uint16_t* colstart = (uint16_t*)(smem + align16((size_t)cap * 4));
    unsigned* cnt = (unsigned*)(smem + align16(align16((size_t)cap * 4) + (size_t)(kGridCols + 1) * 2));
    grid_sort<kSeqGridThreads>(pb, skey, cnt);
    if (st) st[2] = wall_clock64();
    unsigned* gkey = (unsigned*)(gb + gl.skey);
    float2* sxy = (float2*)(gb + gl.sxy);
    float* sang = (float*)(gb + gl.sang);
    int* gfmp = (int*)(gb + gl.sfmp);
    uint4* sdesc = (uint4*)(gb + gl.sdesc);
    for (int p = tid; p < n; p += kSeqGridThreads) {
        const unsigned k = skey[p];
        const int i = sk_idx(k);
        const orbx_keypoint kp = ldg(pb.keys + i);
        gkey[p] = k;
        sxy[p] = make_float2(kp.x, kp.y);
        sang[p] = kp.angle;
        gfmp[p] = claim_word(ldg(pb.frame_mp + i), P);
    }
    for (int t = tid; t < 2 * n; t += kSeqGridThreads) {
        const int i = sk_idx(skey[t >> 1]);
        sdesc[t] = ldg((const uint4*)(pb.desc + (size_t)i * 32) + (t & 1));
    }
    if (st) st[4] = wall_clock64();
    build_colstart<kSeqGridThreads>(skey, n, colstart);
    __syncthreads();
    if (st) st[10] = wall_clock64();
    build_octave_runs<kSeqGridThreads>(skey, colstart, noct, (uint16_t*)(gb + gl.bstart), (uint16_t*)(gb + gl.orun),
                                       cnt);
    if (st) st[11] = wall_clock64();
}

constexpr int kSeqScoreThreads = 256;  // 16 queries (4 per wave, one 16-lane row each)
constexpr int kSeqScoreQ = kSeqScoreThreads / kScoreRow;

__global__ __launch_bounds__(kSeqScoreThreads) void k_seq_score(const ProjProblem* __restrict__ probs, int nprob,
                                                                int qblocks, ProjParams P,
                                                                unsigned char* __restrict__ grids, int cap,
                                                                unsigned long long* __restrict__ scratch,
                                                                const long long* __restrict__ scratch_off) {
    // XCD x (= lin % 8) runs problems x, x + 8, ...: a problem's workgroups share its L2
    const int lin = blockIdx.x, x = lin % kXcds, k = lin / kXcds;
    const int j = k / qblocks, blk = k - j * qblocks;
    const int p = x + kXcds * j;
    if (p >= nprob) return;  // whole workgroup: XCD x has fewer problems
    const ProjProblem pb = probs[p];
    const SeqGridLayout gl(cap, P.noct);
    const SortedGrid G = seq_grid(grids + (size_t)p * gl.total, gl, P.noct);
    const int q = blk * kSeqScoreQ + (int)threadIdx.x / kScoreRow;
    if (blk * kSeqScoreQ >= pb.nq) return;  // whole workgroup past the queries
    const QueryReg cur = load_query(pb, min(q, pb.nq - 1));
    const int mp = q < pb.nq ? cur.q.mp : -1;
    unsigned e[kTopK];
    const int* sfmp0 = (const int*)(grids + (size_t)p * gl.total + gl.sfmp);  // the claims before the search
    score_rowk(pb, P, cur, mp >= 0, G, sfmp0, e);
    if ((threadIdx.x & (kScoreRow - 1)) == 0 && q < pb.nq) {
        unsigned long long* g = scratch + scratch_off[p];
        uint4* qk = (uint4*)g;
        int* qmp = (int*)(g + kListWords * (size_t)pb.nq);
        float* qang = (float*)(qmp + pb.nq);
#pragma unroll
        for (int v = 0; v < kListVec; v++)
            qk[kListVec * q + v] = make_uint4(e[4 * v], e[4 * v + 1], e[4 * v + 2], e[4 * v + 3]);
        qmp[q] = claim_word(mp, P);
        qang[q] = cur.q.angle;
    }
}

template <int RT>
__global__ __launch_bounds__(RT) ORBX_COMMIT_ATTR void k_seq_commit(const ProjProblem* __restrict__ probs, ProjParams P,
                                                   unsigned char* __restrict__ grids, int cap,
                                                   unsigned long long* __restrict__ scratch,
                                                   const long long* __restrict__ scratch_off, int use_sdesc) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_hist[kHistoLength];
#ifndef ORBX_NO_REPLAY_PRIO
    // the replay is latency-bound and shares its CU with the extraction's throughput
    // waves: the highest wave priority makes the SIMD's arbiter issue its instructions first
    __builtin_amdgcn_s_setprio(3);
#endif
    const ProjProblem pb = probs[blockIdx.x];
    if (pb.nq < 0) return;  // skipped by the retry pass (k_seq_score's workgroups leave on nq too)
    unsigned long long* st = P.stamps ? P.stamps + kStampWords * blockIdx.x : nullptr;  // diagnostics
    if (st && threadIdx.x == 0) st[13] = wall_clock64();
    const SeqGridLayout gl(cap, P.noct);
    SortedGrid G = seq_grid(grids + (size_t)blockIdx.x * gl.total, gl, P.noct);
    if (!use_sdesc) G.sdesc = nullptr;  // descriptors by keypoint index from the frame
    const float* gang = (const float*)(grids + (size_t)blockIdx.x * gl.total + gl.sang);
    const int tid = threadIdx.x, n = pb.n, nq = pb.nq;
    // LDS: the replay's lists, the claims and the owner map only (8 B per keypoint); the
    // rotation bins read the grid's angles from global memory after the replay
    unsigned* elist = (unsigned*)smem;
    int* sfmp = (int*)(elist + kTopK * RT);
    int* owner = sfmp + n;
    for (int p = tid; p < n; p += RT) {
        sfmp[p] = claim_word(ldg(pb.frame_mp + sk_idx(G.skey[p])), P);
        owner[p] = RT == 64 ? 0x7fffffff : 0;
    }
    if (tid < kHistoLength) s_hist[tid] = 0;
    __syncthreads();
    unsigned long long* g = scratch + scratch_off[blockIdx.x];
    const uint4* qk = (const uint4*)g;
    const int* qmp = (const int*)(g + kListWords * (size_t)nq);
    const float* qang = (const float*)(qmp + nq);
    int* mlist = (int*)(qang + nq);
    int* mbin = mlist + nq;
    if constexpr (RT == 64)
        proj_replay(pb, P, G, sfmp, owner, elist, qk, qmp, qang, mlist, mbin, s_hist,
                    [&](int tpos) { return gang[tpos]; }, st);
    else
        proj_replay_block<RT>(pb, P, G, sfmp, (unsigned*)owner, elist, qk, qmp, qang, mlist, mbin, s_hist,
                              [&](int tpos) { return gang[tpos]; }, st);
    __syncthreads();
    int32_t* out = P.out_mp ? P.out_mp : pb.frame_mp;
    for (int p = tid; p < n; p += RT) out[sk_idx(G.skey[p])] = claim_mp(sfmp[p]);
}

size_t seq_grid_bytes(int cap, int noct) { return SeqGridLayout(cap, noct).total; }

hipError_t launch_stage_copy(const void* src, void* dst, size_t bytes, hipStream_t stream) {
    if (!bytes) return hipSuccess;
    if (bytes % 16 || ((uintptr_t)src | (uintptr_t)dst) % 16 || bytes / 16 > INT_MAX) return hipErrorInvalidValue;
    const int n16 = (int)(bytes / 16);
    const int blocks = (n16 + kStageThreads * kStageUnroll - 1) / (kStageThreads * kStageUnroll);
    hipLaunchKernelGGL(k_stage_copy, dim3(blocks), dim3(kStageThreads), 0, stream, (const uint4*)src, (uint4*)dst, n16);
    return hipGetLastError();
}

// k_seq_commit's dynamic LDS: the replay's lists, then the claims and the owner map
static size_t seq_commit_lds(int cap, int rt) {
    return (size_t)kTopK * rt * 4 + (size_t)cap * 8;
}

// Threads of the replay workgroup: `rt` if given (64, 128, 256, 512 or 1024), else
// ORBX_REPLAY_THREADS, else 256 for a batch (four waves: configs[4] 93.4-94.2k -> 93.8-95.2k
// frames/s and configs[1] 217.7-219.0k -> 222.3-223.8k against one wave; 1024 threads is
// slower in both, its iterations cost more than the chains it shortens; r05q: 128 and 512
// slower too, configs[4] 108.7-109.8k -> 105.7k / 104.9k) and one wave for a single
// problem (the drop-in host calls: their scenes' conflict chains run across the whole
// chunk, 90 iterations of ~1.9 us at 256 against 109 of ~1.2 us at 64 for a12).
static int replay_threads(int rt, int nprob) {
    if (rt != 64 && rt != 128 && rt != 256 && rt != 512 && rt != 1024) {
        rt = tuning(Tune::ReplayThreads, 0);
    }
    if (rt != 64 && rt != 128 && rt != 256 && rt != 512 && rt != 1024) rt = nprob == 1 ? 64 : 256;
    return rt;
}

static hipError_t launch_seq_commit(int rt, const ProjProblem* d_probs, int nprob, const ProjParams& P,
                                    unsigned char* grids, int cap, unsigned long long* scratch,
                                    const long long* d_scratch_off, int use_sdesc, hipStream_t stream) {
    rt = replay_threads(rt, nprob);
    const size_t lds = seq_commit_lds(cap, rt);
    const void* fn = rt == 64    ? (const void*)k_seq_commit<64>
                     : rt == 128 ? (const void*)k_seq_commit<128>
                     : rt == 256 ? (const void*)k_seq_commit<256>
                     : rt == 512 ? (const void*)k_seq_commit<512>
                                 : (const void*)k_seq_commit<1024>;
    if (lds > 150 * 1024) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    void* args[] = {(void*)&d_probs, (void*)&P, (void*)&grids, (void*)&cap, (void*)&scratch, (void*)&d_scratch_off,
                    (void*)&use_sdesc};
    return hipLaunchKernel(fn, dim3(nprob), dim3(rt), args, lds, stream);
}

hipError_t launch_seq_split(const ProjProblem* d_probs, int nprob, const ProjParams& P, unsigned char* grids,
                            int cap, unsigned long long* scratch, const long long* d_scratch_off, hipStream_t stream,
                            int qcap, int replay_rt, const void* stage_src, void* stage_dst, size_t stage_bytes) {
    if (nprob <= 0) return hipSuccess;
    if (stage_bytes && (nprob != 1 || !stage_src || !stage_dst || stage_bytes % 16 || stage_bytes / 16 > INT_MAX))
        return hipErrorInvalidValue;
    const int n16 = (int)(stage_bytes / 16);
    if (cap <= 0 || cap >= 8192) return hipErrorInvalidValue;  // 13-bit keypoint positions
    if (qcap <= 0) qcap = cap;
    if (P.noct < 1 || P.noct > 32) return hipErrorInvalidValue;
    const size_t scr = octave_runs_scratch(P.noct) > kGridSortScratch ? octave_runs_scratch(P.noct) : kGridSortScratch;
    const size_t lds_grid = align16(align16((size_t)cap * 4) + (size_t)(kGridCols + 1) * 2) + scr;
    // a few problems (the drop-in host calls): 1024 threads per grid, the sort is then on
    // the call's critical path (28 -> ~10 us at C1); a batch: 256, beside the extraction
    const bool wide = nprob < 32;
    const void* gfn = wide ? (const void*)k_seq_grid<1024> : (const void*)k_seq_grid<kSeqGridThreads>;
    if (lds_grid > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(gfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_grid);
        if (e != hipSuccess) return e;
    }
    const uint4* ssrc = (const uint4*)stage_src;
    uint4* sdst = (uint4*)stage_dst;
    if (n16 > 0) {
        const hipError_t ce = launch_stage_copy(ssrc, sdst, (size_t)n16 * 16, stream);
        if (ce != hipSuccess) return ce;
    }
    if (wide)
        hipLaunchKernelGGL(k_seq_grid<1024>, dim3(nprob), dim3(1024), lds_grid, stream, d_probs, P, grids, cap, P.noct,
                           P.stamps);
    else
        hipLaunchKernelGGL(k_seq_grid<kSeqGridThreads>, dim3(nprob), dim3(kSeqGridThreads), lds_grid, stream, d_probs,
                           P, grids, cap, P.noct, P.stamps);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int qblocks = (qcap + kSeqScoreQ - 1) / kSeqScoreQ;
    const int per_xcd = (nprob + kXcds - 1) / kXcds;
    hipLaunchKernelGGL(k_seq_score, dim3(kXcds * per_xcd * qblocks), dim3(kSeqScoreThreads), 0, stream, d_probs,
                       nprob, qblocks, P, grids, cap, scratch, d_scratch_off);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_seq_commit(replay_rt, d_probs, nprob, P, grids, cap, scratch, d_scratch_off, 1, stream);
}

// Batched TrackWithMotionModel matching over a device-resident sequence: problem p
// matches frame p+1 (CurrentFrame) against frame p (LastFrame).  Keypoint i of the last
// frame carries MapPoint id i (Observations() > 0) at mp_pos, or, without mp_pos, at
// depth `depth` on its viewing ray; has_mp masks keypoints without one (or outliers).
// Projection, the forward / backward octave ranges and query construction follow
// SearchByProjection(Frame&, const Frame&, th, bMono) (ORBmatcher.cc:1620-1701).  One
// thread per last-frame keypoint slot.
__global__ __launch_bounds__(256) void k_seq_build(SeqArgs A, ProjQuery* __restrict__ queries,
                                                   ProjProblem* __restrict__ probs,
                                                   long long* __restrict__ scratch_off) {
    const int p = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int nlast = A.n[p];
    // the retry pass (TrackWithMotionModel, Tracking.cc:988-994): only the pairs whose first
    // search found fewer than retry_below matches are searched again, from an empty
    // mvpMapPoints; the others keep the first search's results (problem nq = -1: every later
    // kernel's workgroup leaves at once).  This launch never writes nmatches in the retry
    // pass, so every thread of a pair reads the same gate.
    const bool active = !A.retry_below || A.nmatches[p + 1] < A.retry_below;
    if (i == 0) {
        ProjProblem pb{};
        pb.keys = A.kps + (size_t)(p + 1) * A.cap;
        pb.desc = A.desc + (size_t)(p + 1) * A.cap * 32;
        pb.u_right = A.u_right ? A.u_right + (size_t)(p + 1) * A.cap : nullptr;
        pb.frame_mp = A.cur_mp + (size_t)(p + 1) * A.cap;
        pb.n = A.n[p + 1] < A.cap ? A.n[p + 1] : A.cap;
        pb.q = queries + (size_t)p * A.cap;
        pb.qdesc = A.desc + (size_t)p * A.cap * 32;
        pb.nq = !active ? -1 : (nlast < A.cap ? nlast : A.cap);
        pb.min_x = A.min_x;
        pb.min_y = A.min_y;
        pb.inv_w = (float)kGridCols / (A.max_x - A.min_x);
        pb.inv_h = (float)kGridRows / (A.max_y - A.min_y);
        pb.nmatches = A.nmatches + p + 1;
        probs[p] = pb;
        scratch_off[p] = (long long)p * kProjScratchWords * A.cap;
    }
    if (i >= A.cap || !active) return;
    // the outputs' initial state (no match), here rather than in two memsets: fewer
    // launches on a stream that runs beside the extraction (the retry pass: mvpMapPoints
    // emptied again, Tracking.cc:990-991; its count is the replay's to write)
    A.cur_mp[(size_t)(p + 1) * A.cap + i] = -1;
    if (!A.retry_below) {
        if (p == 0) A.cur_mp[i] = -1;
        if (i == 0) A.nmatches[p + 1] = 0;
        if (p == 0 && i == 0) A.nmatches[0] = 0;
    }
    ProjQuery q{};
    q.mp = -1;
    const size_t slot = (size_t)p * A.cap + i;
    if (i < nlast && !(A.has_mp && !A.has_mp[slot])) {
        const orbx_keypoint kp = A.kps[slot];
        const float* Tl = A.Tcw + 12 * (size_t)p;
        const float* Tc = A.Tcw + 12 * (size_t)(p + 1);
        float Xw[3];
        if (A.mp_pos) {
            for (int c = 0; c < 3; c++) Xw[c] = A.mp_pos[3 * slot + c];
        } else {
            // MapPoint: last-frame camera point on the keypoint ray, to world: Xw = Rl^T (Xc - tl)
            const float z = A.depth;
            const float Xc[3] = {(kp.x - A.cx) / A.fx * z, (kp.y - A.cy) / A.fy * z, z};
            for (int c = 0; c < 3; c++)
                Xw[c] = Tl[c] * (Xc[0] - Tl[3]) + Tl[4 + c] * (Xc[1] - Tl[7]) + Tl[8 + c] * (Xc[2] - Tl[11]);
        }
        // twc = -Rcw^T tcw; tlc = Rlw*twc + tlw (cc:1637-1651), float products left to right
        float twc[3];
        for (int c = 0; c < 3; c++) twc[c] = -(Tc[c] * Tc[3] + Tc[4 + c] * Tc[7] + Tc[8 + c] * Tc[11]);
        const float tlcz = Tl[8] * twc[0] + Tl[9] * twc[1] + Tl[10] * twc[2] + Tl[11];
        const bool bForward = tlcz > A.b && !A.mono;
        const bool bBackward = -tlcz > A.b && !A.mono;
        float x3Dc[3];
        for (int r = 0; r < 3; r++)
            x3Dc[r] = Tc[4 * r] * Xw[0] + Tc[4 * r + 1] * Xw[1] + Tc[4 * r + 2] * Xw[2] + Tc[4 * r + 3];
        const float invzc = (float)(1.0 / (double)x3Dc[2]);
        // fused as g++ -O3 -march=native builds the reference (H4)
        const float u = fmaf(A.fx * x3Dc[0], invzc, A.cx);
        const float v = fmaf(A.fy * x3Dc[1], invzc, A.cy);
        if (!(invzc < 0) && !(u < A.min_x || u > A.max_x) && !(v < A.min_y || v > A.max_y)) {
            const int o = kp.octave;
            q.u = u;
            q.v = v;
            q.ur = fmaf(-A.bf, invzc, u);
            q.r = A.th * A.scale[o];
            q.er_max = q.r;
            if (bForward) {  // GetFeaturesInArea(u, v, radius, nLastOctave)
                q.min_level = o;
                q.max_level = -1;
            } else if (bBackward) {  // (u, v, radius, 0, nLastOctave)
                q.min_level = 0;
                q.max_level = o;
            } else {  // (u, v, radius, nLastOctave-1, nLastOctave+1)
                q.min_level = o - 1;
                q.max_level = o + 1;
            }
            q.post_min = -1;
            q.post_max = -1;
            q.mp = A.global_ids ? (int)slot : i;
            q.angle = kp.angle;
        }
    }
    queries[slot] = q;
}

// ---- Tracking::SearchLocalPoints (Tracking.cc:1280-1336) over a batch of Frames: one
// 1024-thread workgroup per frame builds that frame's SearchByProjection problem.
//   1. mCurrentFrame.mvpMapPoints: a bad MapPoint is set to NULL, the others are marked
//      as seen (mnLastFrameSeen, mbTrackInView = false) -- an LDS hash set of their ids;
//   2. every local MapPoint (mvpLocalMapPoints order) that is neither seen nor bad goes
//      through Frame::IsInFrustum(pMP, 0.5) (Frame.cc:412-477); those in view become the
//      queries of SearchByProjection(F, vpLocalMapPoints, th) (ORBmatcher.cc:61-173), in
//      list order, with r = RadiusByViewingCos(viewCos) (* th when th != 1) *
//      mvScaleFactors[nPredictedLevel] and the levels [nPredictedLevel-1, nPredictedLevel].
// The search itself is the projection matcher's (a11 semantics: Observations() blocking,
// the ratio test on equal levels).  Queries not in view keep their slot with mp = -1.
constexpr int kLocalThreads = 1024;

__device__ __forceinline__ unsigned local_hash(int id, int mask) {
    return ((unsigned)id * 2654435761u) & (unsigned)mask;
}

__global__ __launch_bounds__(kLocalThreads) void k_local_build(LocalArgs A, ProjQuery* __restrict__ queries,
                                                               uint8_t* __restrict__ qdesc,
                                                               ProjProblem* __restrict__ probs,
                                                               long long* __restrict__ scratch_off) {
    extern __shared__ int hset[];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int mask = A.hash_size - 1;
    const int n = A.n[b] < A.cap ? A.n[b] : A.cap;
    int32_t* fmp = A.frame_mp + (size_t)b * A.cap;
    for (int t = tid; t < A.hash_size; t += kLocalThreads) hset[t] = -1;
    __syncthreads();
    for (int i = tid; i < n; i += kLocalThreads) {
        const int mp = fmp[i];
        if (mp < 0) continue;
        // an id outside the MapPoint table (a caller error) is dropped like a NULL entry:
        // never read past the table (orbx.h, orbx_search_local_points_device)
        if ((unsigned)mp >= (unsigned)A.nmp || (A.bad && A.bad[mp])) {  // Tracking.cc:1288-1290
            fmp[i] = -1;
            continue;
        }
        unsigned h = local_hash(mp, mask);
        while (true) {  // open addressing; a frame holds at most cap < hash_size / 2 ids
            const int old = atomicCAS(&hset[h], -1, mp);
            if (old == -1 || old == mp) break;
            h = (h + 1) & (unsigned)mask;
        }
    }
    __syncthreads();
    const int lo = A.local_off[b], hi = A.local_off[b + 1];
    const float* T = A.Tcw + 12 * (size_t)b;
    float Ow[3];  // mOw = -Rcw^T tcw
    for (int c = 0; c < 3; c++) Ow[c] = -(T[c] * T[3] + T[4 + c] * T[7] + T[8 + c] * T[11]);
    const bool bFactor = A.th != 1.0f;  // ORBmatcher.cc:66
    for (int j = lo + tid; j < hi; j += kLocalThreads) {
        const int mp = A.local_ids[j];
        ProjQuery q{};
        q.mp = -1;
        bool in_view = (unsigned)mp < (unsigned)A.nmp && !(A.bad && A.bad[mp]);
        if (in_view) {  // pMP->mnLastFrameSeen == mCurrentFrame.mnId (Tracking.cc:1306-1307)
            unsigned h = local_hash(mp, mask);
            while (true) {
                const int v = hset[h];
                if (v == mp) {
                    in_view = false;
                    break;
                }
                if (v == -1) break;
                h = (h + 1) & (unsigned)mask;
            }
        }
        float u = 0.f, v = 0.f, ur = 0.f, viewCos = 0.f;
        int pred = 0;
        if (in_view) {  // Frame::IsInFrustum (Frame.cc:412-477)
            const float* P = A.pos + 3 * (size_t)mp;
            float Pc[3];
            for (int r = 0; r < 3; r++) Pc[r] = T[4 * r] * P[0] + T[4 * r + 1] * P[1] + T[4 * r + 2] * P[2] + T[4 * r + 3];
            in_view = !(Pc[2] < 0.0f);
            if (in_view) {
                const float invz = 1.0f / Pc[2];
                u = fmaf(A.fx * Pc[0], invz, A.cx);  // fused like the reference's build (H4)
                v = fmaf(A.fy * Pc[1], invz, A.cy);
                ur = fmaf(-A.bf, invz, u);
                in_view = !(u < A.min_x || u > A.max_x) && !(v < A.min_y || v > A.max_y);
            }
            if (in_view) {
                const float maxDistance = 1.2f * A.max_distance[mp];
                const float minDistance = 0.8f * A.min_distance[mp];
                float PO[3];
                for (int c = 0; c < 3; c++) PO[c] = P[c] - Ow[c];
                double ss = 0.0;  // cv::norm: squares in double
                for (int c = 0; c < 3; c++) ss += (double)PO[c] * (double)PO[c];
                const float dist = (float)sqrt(ss);
                in_view = !(dist < minDistance || dist > maxDistance);
                if (in_view) {
                    const float* Pn = A.normal + 3 * (size_t)mp;
                    double dot = 0.0;  // Mat::dot in double
                    for (int c = 0; c < 3; c++) dot += (double)PO[c] * (double)Pn[c];
                    viewCos = (float)(dot / (double)dist);
                    in_view = !(viewCos < A.cos_limit);
                    if (in_view) {  // MapPoint::PredictScale(dist, Frame*) (MapPoint.cc:494-509)
                        const float ratio = A.max_distance[mp] / dist;
                        int ns = (int)ceil(log((double)ratio) / (double)A.log_scale);
                        pred = ns < 0 ? 0 : (ns >= A.nlevels ? A.nlevels - 1 : ns);
                    }
                }
            }
        }
        if (in_view) {
            float r = (double)viewCos > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos, ORBmatcher.cc:176-183
            if (bFactor) r *= A.th;
            q.u = u;
            q.v = v;
            q.ur = ur;
            q.r = r * A.scale[pred];
            q.er_max = r * A.scale[pred];
            q.min_level = pred - 1;
            q.max_level = pred;
            q.post_min = -1;
            q.post_max = -1;
            q.mp = mp;
            q.angle = 0.f;
            const uint4* src = (const uint4*)(A.mdesc + (size_t)mp * 32);
            uint4* dst = (uint4*)(qdesc + (size_t)j * 32);
            dst[0] = src[0];
            dst[1] = src[1];
        }
        queries[j] = q;
    }
    if (tid == 0) {
        ProjProblem pb{};
        pb.keys = A.kps + (size_t)b * A.cap;
        pb.desc = A.desc + (size_t)b * A.cap * 32;
        pb.u_right = A.u_right ? A.u_right + (size_t)b * A.cap : nullptr;
        pb.frame_mp = fmp;
        pb.n = n;
        pb.q = queries + lo;
        pb.qdesc = qdesc + (size_t)lo * 32;
        pb.nq = hi - lo;
        pb.min_x = A.min_x;
        pb.min_y = A.min_y;
        pb.inv_w = (float)kGridCols / (A.max_x - A.min_x);
        pb.inv_h = (float)kGridRows / (A.max_y - A.min_y);
        pb.nmatches = A.nmatches + b;
        probs[b] = pb;
        scratch_off[b] = (long long)lo * kProjScratchWords;
    }
}

hipError_t launch_local_build(const LocalArgs& A, int batch, ProjQuery* queries, uint8_t* qdesc, ProjProblem* probs,
                              long long* scratch_off, hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    if (A.hash_size < 2 * A.cap || (A.hash_size & (A.hash_size - 1)) || A.hash_size > 16384)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_local_build, dim3(batch), dim3(kLocalThreads), (size_t)A.hash_size * 4, stream, A, queries,
                       qdesc, probs, scratch_off);
    return hipGetLastError();
}

hipError_t launch_seq_build(const SeqArgs& A, int npairs, ProjQuery* queries, ProjProblem* probs,
                            long long* scratch_off, hipStream_t stream) {
    if (npairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_seq_build, dim3((A.cap + 255) / 256, npairs), dim3(256), 0, stream, A, queries, probs,
                       scratch_off);
    return hipGetLastError();
}

hipError_t launch_proj_search(const ProjProblem* d_probs, int nprob, const ProjParams& P, unsigned long long* scratch,
                              const long long* d_scratch_off, int max_n, int max_nq, hipStream_t stream, bool small,
                              bool tiny, bool lean, unsigned char* split_grids) {
    if (nprob <= 0) return hipSuccess;
    if (max_n >= 8192) return hipErrorInvalidValue;  // 13-bit keypoint positions
    if (P.noct < 1 || P.noct > 32) return hipErrorInvalidValue;
    const size_t limit = 160 * 1024 - 256;  // minus the static histogram
    // Fast: LDS-resident descriptors (the scoring loads), then LDS-resident query state,
    // 1024 threads.  Small (meant to run beside other kernels): neither, 256 threads.
    small = small || tiny;
    // lean: 1024 threads, but only the grid and the claims in LDS (descriptors and query
    // state in global memory) -- the form that shares a CU best with other kernels
    bool dlds = !small && !lean, qlds = !small && !lean;
    if (dlds && ProjLds(max_n, max_nq, true, true, P.noct).total > limit) {
        qlds = false;
        if (ProjLds(max_n, max_nq, true, false, P.noct).total > limit) {
            dlds = false;
            qlds = ProjLds(max_n, max_nq, false, true, P.noct).total <= limit;
        }
    }
    if (split_grids) {  // lean scoring kernel + k_seq_commit
        if (small) return hipErrorInvalidValue;
        dlds = qlds = false;
    }
    const size_t lds = ProjLds(max_n, max_nq, dlds, qlds, P.noct, split_grids == nullptr,
                               !(split_grids && kSplitSxyGlobal)).total;
    if (lds > limit) return hipErrorInvalidValue;
    const void* fn;
    const int nt = tiny ? kProjThreadsTiny : (small ? kProjThreadsSmall : (split_grids ? kSplitScoreThreads : kProjThreads));
    if (tiny)
        fn = (const void*)k_proj_search<false, false, kProjThreadsTiny>;
    else if (small)
        fn = (const void*)k_proj_search<false, false, kProjThreadsSmall>;
    else if (split_grids)
        fn = (const void*)k_proj_search<false, false, kSplitScoreThreads, true>;
    else
        fn = qlds ? (dlds ? (const void*)k_proj_search<true, true, kProjThreads>
                          : (const void*)k_proj_search<true, false, kProjThreads>)
                  : (dlds ? (const void*)k_proj_search<false, true, kProjThreads>
                          : (const void*)k_proj_search<false, false, kProjThreads>);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    int gcap = max_n;
    void* args[] = {(void*)&d_probs, (void*)&P, (void*)&scratch, (void*)&d_scratch_off, (void*)&split_grids,
                    (void*)&gcap};
    hipError_t e = hipLaunchKernel(fn, dim3(nprob), dim3(nt), args, lds, stream);
    if (e != hipSuccess || !split_grids) return e;
    return launch_seq_commit(0, d_probs, nprob, P, split_grids, max_n, scratch, d_scratch_off, 0, stream);
}

// ------------------------------------------------------------------ triangulation

// One query of SearchForTriangulation = one unmatched KF1 keypoint inside a vocabulary
// node shared with KF2 (ORBmatcher.cc:886-1019), in the reference's visiting order.
// K lanes per query (K = 16: four queries per wave, a shared node's list holds a few
// to a few tens of KF2 keypoints; K = 64: the whole wave on one query).  Returns the
// group's best as a 32-bit key dist << 26 | (2^26 - 1 - offset in the node list): the
// minimum is the smallest distance, the last position on ties (the reference replaces
// its best on dist <= bestDist); 0xffffffff = none.  `valid` false: no query for this
// group.  Must be called with the whole wave active.
template <int K>
__device__ unsigned score_tri_group(const TriProblem& pb, const TriQuery& Q, bool valid, const uint8_t* matched2) {
    static_assert(K == 16 || K == 64, "a DPP row or a wave");
    const int r = threadIdx.x & (K - 1);
    unsigned best = 0xffffffffu;
    if (valid && Q.beg < Q.end) {  // empty range: no shared node (batched tables: filtered queries)
        const orbx_keypoint kp1 = ldg(pb.keys1 + Q.idx1);
        const ulonglong2* d1 = (const ulonglong2*)(pb.desc1 + (size_t)Q.idx1 * 32);
        const ulonglong2 e0 = ldg(d1), e1 = ldg(d1 + 1);
        const unsigned long long q0 = e0.x, q1 = e0.y, q2 = e1.x, q3 = e1.y;
        // epipolar line of kp1 in KF2 (CheckDistEpipolarLine, ORBmatcher.cc:186-213)
        const float* F = pb.F12;
        // fused as g++ -O3 -march=native builds the reference: the first product of each
        // sum goes into an FMA (H4)
        const float a = fmaf(kp1.x, F[0], kp1.y * F[3]) + F[6];
        const float b = fmaf(kp1.x, F[1], kp1.y * F[4]) + F[7];
        const float c = fmaf(kp1.x, F[2], kp1.y * F[5]) + F[8];
        for (int p = Q.beg + r; p < Q.end; p += K) {
            const int idx2 = ldg(pb.fv2_idx + p);
            if (matched2[idx2] || ldg(pb.has_mp2 + idx2)) continue;
            const bool stereo2 = pb.u_right2 && ldg(pb.u_right2 + idx2) >= 0;
            if (pb.only_stereo && !stereo2) continue;
            const ulonglong2* t = (const ulonglong2*)(pb.desc2 + (size_t)idx2 * 32);
            const ulonglong2 t0 = ldg(t), t1 = ldg(t + 1);
            const int dist = __popcll(q0 ^ t0.x) + __popcll(q1 ^ t0.y) + __popcll(q2 ^ t1.x) + __popcll(q3 ^ t1.y);
            if (dist > 50) continue;  // TH_LOW; the running bestDist bound is applied by the key order
            const orbx_keypoint kp2 = ldg(pb.keys2 + idx2);
            if (!Q.stereo1 && !stereo2) {
                const float distex = pb.ex - kp2.x;
                const float distey = pb.ey - kp2.y;
                if (fmaf(distex, distex, distey * distey) < 100 * ldg(pb.scale2 + kp2.octave)) continue;
            }
            const float num = fmaf(a, kp2.x, b * kp2.y) + c;
            const float den = fmaf(a, a, b * b);
            if (den == 0) continue;
            const float dsqr = num * num / den;
            if (!((double)dsqr < 3.84 * (double)ldg(pb.sigma2_2 + kp2.octave))) continue;
            const unsigned key = ((unsigned)dist << 26) | (0x3ffffffu - (unsigned)(p - Q.beg));
            best = key < best ? key : best;
        }
    }
    if (K == 16) return row_min_u32(best);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = umin_(best, (unsigned)__shfl_xor((int)best, o));
    return best;
}

// The 64-bit form the commit reads: dist << 32 | (0xffffffff - offset), or kNoKey.
__device__ __forceinline__ unsigned long long tri_key64(unsigned k32) {
    if (k32 == 0xffffffffu) return kNoKey;
    return ((unsigned long long)(k32 >> 26) << 32) | (0xffffffffu - (0x3ffffffu - (k32 & 0x3ffffffu)));
}

__device__ void score_tri(const TriProblem& pb, const TriQuery& Q, const uint8_t* matched2,
                          unsigned long long& best) {
    best = tri_key64(score_tri_group<64>(pb, Q, true, matched2));
}

// 16 waves score the queries (each scan is a chain of dependent gathers); wave 0 then
// replays the greedy commit.
constexpr int kTriThreads = 1024;

__global__ __launch_bounds__(kTriThreads) void k_triangulation(const TriProblem* __restrict__ probs,
                                                       unsigned long long* __restrict__ scratch) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_hist[kHistoLength];
    const TriProblem pb = probs[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint8_t* matched2 = smem;  // vbMatched2, n2 bytes
    int* owner = (int*)(smem + ((pb.n2 + 15) & ~15));  // lowest lane of a commit round wanting KF2 keypoint i
    int* mlist = owner + pb.n2;
    int* mbin = mlist + pb.nq;
    for (int i = tid; i < pb.n2; i += kTriThreads) {
        matched2[i] = 0;
        owner[i] = 0x7fffffff;
    }
    if (tid < kHistoLength) s_hist[tid] = 0;
    __syncthreads();
    unsigned long long* keys = scratch + pb.scratch_off;
    // candidate scans: all waves, four queries per wave (16-lane rows)
    for (int q0 = wave * 4; q0 < pb.nq; q0 += kTriThreads / 16) {
        const int q = q0 + (lane >> 4);
        const bool valid = q < pb.nq;
        const unsigned best = score_tri_group<16>(pb, ldg(pb.q + (valid ? q : q0)), valid, matched2);
        if (valid && (lane & 15) == 0) keys[q] = tri_key64(best);
    }
    __syncthreads();
    if (wave == 0) {
        // The greedy commit (cc:985-990) in query order, 64 queries per chunk: lane i
        // prefetches query q0+i's record, pre-scored best, candidate and angles, and the
        // sequential walk reads them back by v_readlane, so only a claimed best (a
        // re-score against the current vbMatched2) touches global memory.
        int nrec = 0;
        const float factor = kHistoLength / 360.0f;
        for (int q0 = 0; q0 < pb.nq; q0 += 64) {
            const int ql = q0 + lane;
            int l_idx1 = 0, l_idx2 = -1;
            unsigned long long l_best = kNoKey;
            float l_a1 = 0.f, l_a2 = 0.f;
            if (ql < pb.nq) {
                const TriQuery Q = ldg(pb.q + ql);
                l_idx1 = Q.idx1;
                l_best = keys[ql];
                if (l_best != kNoKey) {
                    l_idx2 = ldg(pb.fv2_idx + Q.beg + (int)(0xffffffffu - (unsigned)(l_best & 0xffffffffu)));
                    l_a2 = ldg(&pb.keys2[l_idx2].angle);
                }
                if (Q.idx1 >= 0) l_a1 = ldg(&pb.keys1[Q.idx1].angle);
            }
            // Rounds over the chunk: a lane's pre-scored best is still its answer unless an
            // earlier query took that keypoint (vbMatched2) or an earlier lane of this round
            // wants it too (owner map).  All lanes before the first such conflict commit at
            // once; the conflicting query is re-scored against the current vbMatched2 (now
            // holding every earlier claim) and commits alone; the next round starts after it.
            int start = 0;
            while (true) {
                const bool act = lane >= start && ql < pb.nq && l_idx1 >= 0 && l_idx2 >= 0;
                const bool taken = act && matched2[l_idx2];
                if (act && !taken) atomicMin(&owner[l_idx2], lane);
                const bool dup = act && !taken && owner[l_idx2] < lane;
                if (act && !taken) owner[l_idx2] = 0x7fffffff;
                const unsigned long long cm = __ballot(taken || dup);
                const int f = cm ? __ffsll((long long)cm) - 1 : 64;
                const bool com = act && lane < f;
                if (com) {
                    pb.matches12[l_idx1] = l_idx2;
                    matched2[l_idx2] = 1;
                }
                if (pb.check_ori) {
                    const unsigned long long comm = __ballot(com);
                    if (com) {
                        float rot = l_a1 - l_a2;
                        if (rot < 0.0f) rot += 360.0f;
                        int bin = (int)roundf(rot * factor);
                        if (bin == kHistoLength) bin = 0;
                        const int r = nrec + __popcll(comm & ((1ull << lane) - 1ull));
                        mlist[r] = l_idx1;
                        mbin[r] = bin;
                        atomicAdd(&s_hist[bin], 1);
                    }
                    nrec += __popcll(comm);
                }
                if (f >= 64) break;
                wave_lds_fence();
                // query q0 + f: re-score against the current claims, commit alone
                const TriQuery Q = ldg(pb.q + q0 + f);
                unsigned long long best;
                score_tri(pb, Q, matched2, best);
                const int idx1 = __builtin_amdgcn_readlane(l_idx1, f);
                const int idx2 = best != kNoKey
                                     ? ldg(pb.fv2_idx + Q.beg + (int)(0xffffffffu - (unsigned)(best & 0xffffffffu)))
                                     : -1;
                if (lane == f) l_idx2 = -1;  // resolved
                if (idx2 >= 0) {
                    if (lane == 0) {
                        pb.matches12[idx1] = idx2;
                        matched2[idx2] = 1;
                    }
                    if (pb.check_ori) {
                        float rot = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(l_a1), f)) -
                                    pb.keys2[idx2].angle;
                        if (rot < 0.0f) rot += 360.0f;
                        int bin = (int)roundf(rot * factor);
                        if (bin == kHistoLength) bin = 0;
                        if (lane == 0) {
                            mlist[nrec] = idx1;
                            mbin[nrec] = bin;
                            s_hist[bin]++;
                        }
                        nrec++;
                    }
                }
                start = f + 1;
                wave_lds_fence();
            }
            wave_lds_fence();
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        if (pb.check_ori) {
            int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
            for (int i = 0; i < kHistoLength; i++) {
                const int s = s_hist[i];
                if (s > max1) {
                    max3 = max2; max2 = max1; max1 = s;
                    ind3 = ind2; ind2 = ind1; ind1 = i;
                } else if (s > max2) {
                    max3 = max2; max2 = s;
                    ind3 = ind2; ind2 = i;
                } else if (s > max3) {
                    max3 = s;
                    ind3 = i;
                }
            }
            if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
            else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
            for (int m = lane; m < nrec; m += 64) {
                const int b = mbin[m];
                if (b != ind1 && b != ind2 && b != ind3) pb.matches12[mlist[m]] = -1;
            }
        }
        if (pb.pairs_out) {
            // vMatchedPairs (cc:1045-1053): vMatches12 compacted in idx1 order, 64 at a time
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            int cnt = 0;
            for (int base = 0; base < pb.n1; base += 64) {
                const int i = base + lane;
                const int v = i < pb.n1 ? pb.matches12[i] : -1;
                const unsigned long long mask = __ballot(v >= 0);
                const int pre = __popcll(mask & ((1ull << lane) - 1ull));
                if (v >= 0) {
                    pb.pairs_out[2 * (cnt + pre)] = i;
                    pb.pairs_out[2 * (cnt + pre) + 1] = v;
                }
                cnt += __popcll(mask);
            }
            if (lane == 0) *pb.npairs_out = cnt;
        }
    }
}

// Batched form: one workgroup per (KF1, KF2) pair builds that pair's query table and
// problem record on the device from the keyframe tables (the FeatureVector merge of
// ORBmatcher.cc:886-1019).  Query q is KF1's q-th FeatureVector entry, so the table is in
// the reference's visiting order (nodes ascending, keypoints in node-list order); an
// entry whose node KF2 lacks, whose keypoint already has a MapPoint (cc:905-909) or that
// fails bOnlyStereo (cc:913-916) gets an empty candidate range.
constexpr int kTriSetupThreads = 256;

__global__ __launch_bounds__(kTriSetupThreads) void k_tri_setup(TriBatch tb) {
    const int p = blockIdx.x, tid = threadIdx.x;
    const TriPair pr = tb.pairs[p];
    const TriKF A = tb.kfs[pr.kf1];
    const TriKF B = tb.kfs[pr.kf2];
    const int cap = tb.cap;
    const int n1 = min(max(*A.n, 0), cap), n2 = min(max(*B.n, 0), cap);
    const int nfv1 = min(max(*A.nfv, 0), n1), nfv2 = min(max(*B.nfv, 0), n2);
    int32_t* m12 = tb.matches12 + (size_t)p * cap;
    for (int i = tid; i < cap; i += kTriSetupThreads) m12[i] = -1;
    TriQuery* Q = tb.q + (size_t)p * cap;
    const int nq = min(A.fv_off[nfv1], n1);
    for (int q = tid; q < nq; q += kTriSetupThreads) Q[q] = TriQuery{-1, 0, 0, 0};  // entries no node covers
    __syncthreads();
    for (int j1 = tid; j1 < nfv1; j1 += kTriSetupThreads) {
        const int node = A.fv_node[j1];
        int lo = 0, hi = nfv2;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (B.fv_node[mid] < node) lo = mid + 1;
            else hi = mid;
        }
        const bool shared = lo < nfv2 && B.fv_node[lo] == node;
        const int beg = shared ? B.fv_off[lo] : 0, end = shared ? min(B.fv_off[lo + 1], n2) : 0;
        const int q1 = min(A.fv_off[j1 + 1], nq);
        for (int q = max(A.fv_off[j1], 0); q < q1; q++) {
            int idx1 = A.fv_idx[q];
            TriQuery t;
            t.beg = t.end = 0;
            t.stereo1 = 0;
            if (idx1 < 0 || idx1 >= n1) {
                idx1 = -1;
            } else {
                const bool st1 = A.u_right && A.u_right[idx1] >= 0;
                t.stereo1 = st1 ? 1 : 0;
                if (shared && !A.has_mp[idx1] && (!tb.only_stereo || st1)) {
                    t.beg = beg;
                    t.end = end;
                }
            }
            t.idx1 = idx1;
            Q[q] = t;
        }
    }
    if (tid == 0) {
        TriProblem pb{};
        pb.keys1 = A.keys;
        pb.desc1 = A.desc;
        pb.keys2 = B.keys;
        pb.desc2 = B.desc;
        pb.u_right2 = B.u_right;
        pb.has_mp2 = B.has_mp;
        pb.fv2_idx = B.fv_idx;
        pb.scale2 = tb.scale2;
        pb.sigma2_2 = tb.sigma2_2;
        for (int k = 0; k < 9; k++) pb.F12[k] = pr.F12[k];
        pb.ex = pr.ex;
        pb.ey = pr.ey;
        pb.only_stereo = tb.only_stereo;
        pb.check_ori = tb.check_ori;
        pb.n2 = n2;
        pb.q = Q;
        pb.nq = nq;
        pb.matches12 = m12;
        pb.scratch_off = (long long)p * cap;
        pb.n1 = n1;
        pb.pairs_out = tb.pairs_out + (size_t)p * cap * 2;
        pb.npairs_out = tb.npairs_out + p;
        tb.probs[p] = pb;
    }
}

hipError_t launch_triangulation(const TriProblem* d_probs, int nprob, unsigned long long* scratch, int max_n2,
                                int max_nq, hipStream_t stream) {
    if (nprob <= 0) return hipSuccess;
    const size_t lds = (size_t)((max_n2 + 15) & ~15) + (size_t)max_n2 * 4 + (size_t)max_nq * 8;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)k_triangulation, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_triangulation, dim3(nprob), dim3(kTriThreads), lds, stream, d_probs, scratch);
    return hipGetLastError();
}

hipError_t launch_triangulation_batch(const TriBatch& tb, unsigned long long* scratch, hipStream_t stream) {
    if (tb.npairs <= 0) return hipSuccess;
    if (tb.cap <= 0 || tb.cap > 8192) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_tri_setup, dim3(tb.npairs), dim3(kTriSetupThreads), 0, stream, tb);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_triangulation(tb.probs, tb.npairs, scratch, tb.cap, tb.cap, stream);
}

// ------------------------------------------------------------------ stereo

// Frame::ComputeStereoMatches (Frame.cc:673-885) for B left/right pairs, three launches:
//   k_stereo_index    vRowIndices (cc:693-708) of each pair, restated as a CSR over
//                     (octave, row) plus each row's list size;
//   k_stereo          a 16-lane row per left keypoint: row-band Hamming search, 11x11 SAD over
//                     shifts -5..5 on the pyramid level, parabola fit (cc:720-866);
//   k_stereo_outlier  this fork's outlier pass, which sits inside the iL loop
//                     (cc:868-884, hazard H8): after every iteration that reaches it,
//                     vDistIdx is sorted and entries with dist >= 1.5*1.4*median are
//                     invalidated.
// The row lists hold right keypoints in any order: the search keeps the smallest
// (distance, iR), which is the reference's first-wins `dist < bestDist` over its
// ascending-iR lists.

// Exclusive prefix sum of a[0, n) in place by one workgroup of NT threads (tmp: NT ints
// of LDS); returns the total.  Must be called by all NT threads.
template <int NT>
__device__ int block_exscan_inplace(int* a, int n, int* tmp) {
    const int t = threadIdx.x;
    const int seg = (n + NT - 1) / NT;
    const int b = t * seg, e = min(n, b + seg);
    int sum = 0;
    for (int i = b; i < e; i++) sum += a[i];
    tmp[t] = sum;
    __syncthreads();
    for (int o = 1; o < NT; o <<= 1) {
        const int v = t >= o ? tmp[t - o] : 0;
        __syncthreads();
        tmp[t] += v;
        __syncthreads();
    }
    int run = tmp[t] - sum;  // exclusive prefix of this thread's segment
    const int total = tmp[NT - 1];
    for (int i = b; i < e; i++) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
    return total;
}

// vRowIndices (cc:693-708) restated for a search that keeps the smallest (distance, iR):
// the reference pushes right keypoint iR into the list of every row floor(y - r) ..
// ceil(y + r), r = 2 scale[octave], and a left keypoint at row (int)vL scans that row's
// list, skipping octaves outside levelL +- 1.  Here each right keypoint is listed once,
// under (octave, floor(y)); the search visits, per admissible octave, the few rows whose
// keypoints can cover its row and tests the band exactly -- the same candidate set, without
// the ~7x duplication of the row lists (round 4's k_stereo_rows: one 1024-thread workgroup
// per pair pushing every band row, 0.79 ms per 128 KITTI pairs beside the extraction).
// The reference also needs each row's list size (empty: the left keypoint is skipped,
// cc:728): a difference array over the bands gives it.
constexpr int kStereoIdxThreads = 256;

__global__ __launch_bounds__(kStereoIdxThreads) void k_stereo_index(StereoBatch sb) {
    extern __shared__ __align__(16) int s_idx[];  // cnt [L * rows + 1], then cov [rows + 1]
    __shared__ int s_tmp[kStereoIdxThreads];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int rows = sb.rows, L = sb.nlevels, nb = L * rows;
    int* cnt = s_idx;
    int* cov = s_idx + nb + 1;
    const int nr = min(sb.n_r[b], sb.cap);
    const orbx_keypoint* kr = sb.keys_r + (size_t)b * sb.cap;
    for (int i = tid; i <= nb; i += kStereoIdxThreads) cnt[i] = 0;
    for (int i = tid; i <= rows; i += kStereoIdxThreads) cov[i] = 0;
    __syncthreads();
    for (int iR = tid; iR < nr; iR += kStereoIdxThreads) {
        const orbx_keypoint kp = ldg(kr + iR);
        const int o = min(max(kp.octave, 0), L - 1);
        const int yb = min(max((int)kp.y, 0), rows - 1);
        atomicAdd(&cnt[o * rows + yb], 1);
        // the rows this keypoint's list entries would cover (rows outside the image, which
        // keypoints >= 16 px inside never reach, are dropped)
        const float r = 2.0f * sb.scale[o];  // the clamped octave k_stereo tests the band with
        const int lo = max((int)floorf(kp.y - r), 0), hi = min((int)ceilf(kp.y + r), rows - 1);
        if (lo <= hi) {
            atomicAdd(&cov[lo], 1);
            atomicAdd(&cov[hi + 1], -1);
        }
    }
    __syncthreads();
    const int total = block_exscan_inplace<kStereoIdxThreads>(cnt, nb, s_tmp);
    block_exscan_inplace<kStereoIdxThreads>(cov, rows + 1, s_tmp);  // cov[y + 1]: rows <= y summed
    int32_t* off = sb.row_off + (size_t)b * (nb + 1 + rows);
    for (int i = tid; i < nb; i += kStereoIdxThreads) off[i] = cnt[i];
    if (tid == 0) off[nb] = total;
    for (int y = tid; y < rows; y += kStereoIdxThreads) off[nb + 1 + y] = cov[y + 1];
    __syncthreads();  // every offset read before the cursors below move them
    int32_t* idx = sb.row_idx + (size_t)b * sb.band_cap;
    for (int iR = tid; iR < nr; iR += kStereoIdxThreads) {
        const orbx_keypoint kp = ldg(kr + iR);
        const int o = min(max(kp.octave, 0), L - 1);
        const int yb = min(max((int)kp.y, 0), rows - 1);
        idx[atomicAdd(&cnt[o * rows + yb], 1)] = iR;
    }
}

// One wave per left keypoint of pair blockIdx.y.
// k_stereo: four left keypoints per wave (16-lane rows; round 3, one per wave before:
// KITTI 55.5-55.7k -> 57.9-58.3k stereo frames/s, EuRoC +7 %).  A row
// band holds tens of right keypoints and the SAD window 121 pixels, so a whole wave per
// keypoint left most lanes idle in the band scan's last pass and the SAD's second; here
// a row's 16 lanes share the band scan (key dist << 23 | iR: the smallest distance, then
// the first right keypoint of the row list, as the reference's strict <) and each SAD
// (the 11 shifts' sums by DPP row reductions).  Rows whose keypoint stops early (empty
// band, no match, out-of-image window, border shift, |deltaR| > 1) carry their result
// along with the wave; lane 0 of a row writes it.
__device__ __forceinline__ unsigned row_sum_u32(unsigned v) {
    v += (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false);
    v += (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false);
    return v;
}

__global__ __launch_bounds__(256) void k_stereo(StereoBatch sb) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int gl = lane & 15;
    const int b = blockIdx.y;
    const int base = (blockIdx.x * 4 + wave) * 4;
    const int iL = base + (lane >> 4);
    const int nl = min(sb.n_l[b], sb.cap);
    if (base >= nl) return;  // whole wave
    const bool valid = iL < nl;
    StereoResult res;
    res.reach_sort = 0;
    res.pushed = 0;
    res.dist = 0;
    res.u_right = -1.f;
    res.depth = -1.f;
    const orbx_keypoint kpL = sb.keys_l[(size_t)b * sb.cap + (valid ? iL : base)];
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    const int row = (int)vL;
    const int nb = sb.nlevels * sb.rows;
    const int32_t* roff = sb.row_off + (size_t)b * (nb + 1 + sb.rows);
    const bool listed = row >= 0 && row < sb.rows && roff[nb + 1 + row] > 0;  // !vRowIndices[vL].empty()
    const float minD = 0.f;
    const bool scan = valid && listed && uL - minD >= 0;  // cc:727-735
    const float minU = uL - sb.max_d, maxU = uL - minD;
    const int32_t* ridx = sb.row_idx + (size_t)b * sb.band_cap;
    const orbx_keypoint* kr = sb.keys_r + (size_t)b * sb.cap;
    const uint8_t* dr = sb.desc_r + (size_t)b * sb.cap * 32;
    unsigned best = 0xffffffffu;
    if (scan) {
        const unsigned long long* dl = (const unsigned long long*)(sb.desc_l + ((size_t)b * sb.cap + iL) * 32);
        const unsigned long long q0 = dl[0], q1 = dl[1], q2 = dl[2], q3 = dl[3];
        // octaves levelL - 1 .. levelL + 1 (cc:748-749); per octave o the keypoints whose band
        // [floor(y - r), ceil(y + r)], r = 2 scale[o], covers `row` lie in the rows
        // floor(y) = row - ceil(r) - 1 .. row + ceil(r) + 1, and are tested exactly
        for (int o = max(levelL - 1, 0); o <= min(levelL + 1, sb.nlevels - 1); o++) {
            const float r = 2.0f * sb.scale[o];
            const int R = (int)ceilf(r) + 1;
            const int y0 = max(row - R, 0), y1 = min(row + R, sb.rows - 1);
            const int cbeg = roff[o * sb.rows + y0], cend = roff[o * sb.rows + y1 + 1];
            for (int p = cbeg + gl; p < cend; p += 16) {
                const int iR = ridx[p];
                const orbx_keypoint kpR = kr[iR];
                if ((int)floorf(kpR.y - r) > row || (int)ceilf(kpR.y + r) < row) continue;  // not in vRowIndices[row]
                const float uR = kpR.x;
                if (uR >= minU && uR <= maxU) {
                    const unsigned long long* t = (const unsigned long long*)(dr + (size_t)iR * 32);
                    const int d = __popcll(q0 ^ t[0]) + __popcll(q1 ^ t[1]) + __popcll(q2 ^ t[2]) + __popcll(q3 ^ t[3]);
                    best = umin_(best, ((unsigned)d << 23) | (unsigned)iR);
                }
            }
        }
    }
    best = row_min_u32(best);
    if (scan) res.reach_sort = 1;
    const int bestDist = best == 0xffffffffu ? 100 : (int)(best >> 23);  // starts at TH_HIGH, strict <
    bool sad = scan && bestDist < 75;                                     // thOrbDist = (TH_HIGH + TH_LOW) / 2
    const int w = 5, L = 5;
    float scaleduL = 0.f, scaledvL = 0.f, scaleduR0 = 0.f;
    if (sad) {
        const int bestIdxR = (int)(best & 0x7fffffu);
        const float uR0 = kr[bestIdxR].x;
        const float scaleFactor = sb.inv_scale[levelL];
        scaleduL = roundf(kpL.x * scaleFactor);
        scaledvL = roundf(kpL.y * scaleFactor);
        scaleduR0 = roundf(uR0 * scaleFactor);
        const float iniu = scaleduR0 + L - w;
        const float endu = scaleduR0 + L + w + 1;
        if (iniu < 0 || endu >= sb.level_w[levelL]) {  // cc:810-811
            res.reach_sort = 0;
            sad = false;
        }
    }
    float vd[11];
    int bestDistS = 0x7fffffff, bestincR = 0;
    {
        // level 0 from the caller's frames when the extraction read it in place
        const bool inl = sad && levelL == 0 && sb.l0_l, inr = sad && levelL == 0 && sb.l0_r;
        const int pitch = inl ? sb.l0_pitch_l : (sad ? sb.level_pitch[levelL] : 0);
        const int pitchR = inr ? sb.l0_pitch_r : (sad ? sb.level_pitch[levelL] : 0);
        const uint8_t* IL = inl ? sb.l0_l + (size_t)b * sb.l0_fp_l
                                : sb.pyr_l + (size_t)b * sb.fb_l + (sad ? sb.level_off[levelL] : 0);
        const uint8_t* IR = inr ? sb.l0_r + (size_t)b * sb.l0_fp_r
                                : sb.pyr_r + (size_t)b * sb.fb_r + (sad ? sb.level_off[levelL] : 0);
        const int yl0 = (int)scaledvL - w, xl0 = (int)scaleduL - w;
        int cl = 0;
        int a8[8];
        if (sad) {
            cl = IL[(size_t)(yl0 + w) * pitch + xl0 + w];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int k = gl + 16 * j;
                const int yy = k / 11, xx = k - yy * 11;
                a8[j] = k < 121 ? (int)IL[(size_t)(yl0 + yy) * pitch + xl0 + xx] - cl : 0;
            }
        }
#pragma unroll
        for (int incR = -L; incR <= L; incR++) {
            int acc = 0;
            if (sad) {
                const int xr0 = (int)(scaleduR0 + incR - w);
                const int cr = IR[(size_t)(yl0 + w) * pitchR + xr0 + w];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const int k = gl + 16 * j;
                    if (k < 121) {
                        const int yy = k / 11, xx = k - yy * 11;
                        const int c = (int)IR[(size_t)(yl0 + yy) * pitchR + xr0 + xx] - cr;
                        acc += a8[j] > c ? a8[j] - c : c - a8[j];
                    }
                }
            }
            acc = (int)row_sum_u32((unsigned)acc);
            const float dist = (float)acc;  // cv::norm(IL, IR, NORM_L1) on integer-valued floats
            if (dist < (float)bestDistS) {
                bestDistS = (int)dist;
                bestincR = incR;
            }
            vd[L + incR] = dist;
        }
    }
    if (sad && (bestincR == -L || bestincR == L)) {  // cc:834-835
        res.reach_sort = 0;
        sad = false;
    }
    if (sad) {
        float dist1 = vd[0], dist2 = vd[0], dist3 = vd[0];
#pragma unroll
        for (int k = 0; k < 11; k++) {
            if (k == L + bestincR - 1) dist1 = vd[k];
            if (k == L + bestincR) dist2 = vd[k];
            if (k == L + bestincR + 1) dist3 = vd[k];
        }
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) {  // cc:845-846
            res.reach_sort = 0;
        } else {
            float bestuR = sb.scale[levelL] * (scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < sb.max_d) {
                if (disparity <= 0) {
                    disparity = 0.01f;
                    bestuR = (float)((double)uL - 0.01);
                }
                res.depth = sb.bf / disparity;
                res.u_right = bestuR;
                res.pushed = 1;
                res.dist = bestDistS;
            }
        }
    }
    if (valid && gl == 0) sb.res[(size_t)b * sb.cap + iL] = res;
}


// The in-loop outlier pass (cc:868-884) of one pair per 1024-thread workgroup.
//
// The pass at iteration t marks every pushed entry whose dist >= thDist_t = 1.5f * 1.4f *
// median_t, where median_t is the (s_t / 2)-th smallest dist of the s_t entries pushed
// so far (vDistIdx sorted by (dist, iL)); a marked entry stays -1.  So entry j ends
// invalid iff (float)dist_j >= min over reaching iterations t >= j of thDist_t.
//   1. the pushed (dist, iL) keys are block-sorted: an entry's rank is its position in
//      the reference's sorted vDistIdx at the end of the loop;
//   2. the iterations are cut into 16 chunks, one per wave.  A wave sets the rank bits
//      of the entries pushed before its chunk, finds their (s/2)-th rank, and walks its
//      chunk in order: each push moves the median rank by at most one present rank
//      (nearest set bit), so every reaching iteration's median costs O(1);
//   3. a suffix minimum of thDist over the iterations, then one comparison per entry.
// An empty vDistIdx at a reaching iteration (the reference reads vDistIdx[0] of an
// empty vector there) marks nothing.
constexpr int kStereoOutThreads = 1024;
constexpr int kStereoOutWaves = kStereoOutThreads / 64;

__global__ __launch_bounds__(kStereoOutThreads) void k_stereo_outlier(StereoBatch sb, int n2) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ float s_seg[kStereoOutThreads];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int N = min(sb.n_l[b], sb.cap);
    const StereoResult* R = sb.res + (size_t)b * sb.cap;
    unsigned long long* skey = (unsigned long long*)smem;                   // n2 (sort)
    uint16_t* rank = (uint16_t*)(smem + (size_t)8 * n2);                      // n2
    uint8_t* flag = (uint8_t*)(smem + (size_t)10 * n2);                       // n2: 1 pushed, 2 reaches the pass
    unsigned long long* bits = (unsigned long long*)(smem + (size_t)11 * n2); // per wave n2 / 64 words
    const int nw = n2 >> 6;
    // 1. sort the pushed entries by (dist, iL)
    const int ne = n2 / kSortThreads;
    unsigned long long r[kSortPer];
#pragma unroll
    for (int e = 0; e < kSortPer; e++) {
        r[e] = ~0ull;
        const int i = e * kSortThreads + tid;
        if (e < ne && i < N) {
            const StereoResult x = R[i];
            flag[i] = (uint8_t)((x.pushed ? 1 : 0) | (x.reach_sort ? 2 : 0));
            if (x.pushed) r[e] = ((unsigned long long)(unsigned)x.dist << 32) | (unsigned)i;
        }
    }
    block_bitonic_sort64(r, ne, skey);
    for (int m = tid; m < n2; m += kStereoOutThreads) {
        const unsigned long long k = skey[m];
        if (k != ~0ull) rank[(int)(k & 0xffffffffu)] = (uint16_t)m;
    }
    // sorted dist values (u32) over the first half of the sort buffer, thresholds over the second
    unsigned dv[kSortPer];
#pragma unroll
    for (int e = 0; e < kSortPer; e++)
        if (e < ne) dv[e] = (unsigned)(skey[e * kSortThreads + tid] >> 32);
    __syncthreads();
    unsigned* sdist = (unsigned*)smem;
    float* thr = (float*)(smem + (size_t)4 * n2);
#pragma unroll
    for (int e = 0; e < kSortPer; e++)
        if (e < ne) sdist[e * kSortThreads + tid] = dv[e];
    unsigned long long* W = bits + (size_t)wave * nw;
    for (int w = lane; w < nw; w += 64) W[w] = 0ull;
    __syncthreads();
    // 2. per-wave chunk walk
    const int chunk = (N + kStereoOutWaves - 1) / kStereoOutWaves;
    const int t0 = min(N, wave * chunk), t1 = min(N, t0 + chunk);
    for (int j = lane; j < t0; j += 64)
        if (flag[j] & 1) atomicOr(&W[rank[j] >> 6], 1ull << (rank[j] & 63));
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
    // s = entries pushed before t0; m = rank of the (s / 2)-th of them (order statistic)
    int s = 0;
    for (int w = lane; w < nw; w += 64) s += __popcll(W[w]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    int m = -1;
    if (s > 0) {
        const int k = s >> 1;
        int base = 0;
        for (int w0 = 0; w0 < nw; w0 += 64) {
            const unsigned long long word = w0 + lane < nw ? W[w0 + lane] : 0ull;
            const int c = __popcll(word);
            int incl = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(incl, o);
                if (lane >= o) incl += v;
            }
            const unsigned long long hit = __ballot(base + incl > k);
            if (hit) {
                const int src = __ffsll((long long)hit) - 1;
                if (lane == src) {
                    int need = k - (base + incl - c);  // set bits of this word to skip
                    unsigned long long x = word;
                    while (need-- > 0) x &= x - 1;
                    m = (w0 + lane) * 64 + __ffsll((long long)x) - 1;
                }
                m = __shfl(m, src);
                break;
            }
            base += __shfl(incl, 63);
        }
    }
    if (lane == 0) {
        int kc = s > 0 ? (s >> 1) : 0;
        for (int t = t0; t < t1; t++) {
            const int f = flag[t];
            if (f & 1) {
                const int rt = rank[t];
                W[rt >> 6] |= 1ull << (rt & 63);
                s++;
                if (s == 1) {
                    m = rt;
                    kc = 0;
                } else {
                    if (rt < m) kc++;
                    const int k = s >> 1;
                    if (kc < k) {  // next present rank above m
                        int w = m >> 6;
                        unsigned long long x = (m & 63) == 63 ? 0ull : (W[w] & (~0ull << ((m & 63) + 1)));
                        while (!x) x = W[++w];
                        m = w * 64 + __ffsll((long long)x) - 1;
                        kc++;
                    } else if (kc > k) {  // previous present rank below m
                        int w = m >> 6;
                        unsigned long long x = W[w] & ((1ull << (m & 63)) - 1);
                        while (!x) x = W[--w];
                        m = w * 64 + 63 - __clzll((long long)x);
                        kc--;
                    }
                }
            }
            thr[t] = ((f & 2) && s > 0) ? 1.5f * 1.4f * (float)sdist[m] : __int_as_float(0x7f800000);
        }
    }
    __syncthreads();
    // 3. suffix minimum over t, then the marks
    const int seg = (N + kStereoOutThreads - 1) / kStereoOutThreads;
    const int a = tid * seg, e = min(N, a + seg);
    float mn = __int_as_float(0x7f800000);
    for (int i = e - 1; i >= a; i--) {
        mn = fminf(mn, thr[i]);
        thr[i] = mn;
    }
    s_seg[tid] = mn;
    __syncthreads();
    for (int o = 1; o < kStereoOutThreads; o <<= 1) {
        const float v = tid + o < kStereoOutThreads ? s_seg[tid + o] : __int_as_float(0x7f800000);
        __syncthreads();
        s_seg[tid] = fminf(s_seg[tid], v);
        __syncthreads();
    }
    float* ur = sb.u_right + (size_t)b * sb.cap;
    float* dp = sb.depth + (size_t)b * sb.cap;
    for (int i = tid; i < sb.cap; i += kStereoOutThreads) {
        float u = -1.f, d = -1.f;
        if (i < N && (flag[i] & 1)) {
            const int q = i / seg;
            const float after = q + 1 < kStereoOutThreads ? s_seg[q + 1] : __int_as_float(0x7f800000);
            const float th = fminf(thr[i], after);
            const StereoResult x = R[i];
            if ((float)x.dist < th) {
                u = x.u_right;
                d = x.depth;
            }
        }
        ur[i] = u;
        dp[i] = d;
    }
}

size_t stereo_outlier_lds(int cap) {
    int n2 = kSortThreads;
    while (n2 < cap) n2 <<= 1;
    return (size_t)13 * n2;
}

hipError_t launch_stereo(const StereoBatch& sb, int batch, hipStream_t stream) {
    if (batch <= 0) return hipSuccess;
    if (sb.cap > kSortMaxKeys || sb.rows <= 0 || sb.nlevels < 1 || sb.nlevels > 32) return hipErrorInvalidValue;
    const size_t idx_lds = ((size_t)sb.nlevels * sb.rows + 1 + sb.rows + 1) * 4;
    if (idx_lds > 150 * 1024) return hipErrorInvalidValue;
    if (idx_lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)k_stereo_index, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)idx_lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_stereo_index, dim3(batch), dim3(kStereoIdxThreads), idx_lds, stream, sb);
    hipLaunchKernelGGL(k_stereo, dim3((sb.cap + 15) / 16, batch), dim3(256), 0, stream, sb);
    int n2 = kSortThreads;
    while (n2 < sb.cap) n2 <<= 1;
    const size_t lds = stereo_outlier_lds(sb.cap);
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)k_stereo_outlier, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_stereo_outlier, dim3(batch), dim3(kStereoOutThreads), lds, stream, sb, n2);
    return hipGetLastError();
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
