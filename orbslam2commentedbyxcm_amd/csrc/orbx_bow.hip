// orbx_bow.hip -- vocabulary-node and initialisation matchers:
//   ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...)      ORBmatcher.cc:228-392
//   ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, ...)   ORBmatcher.cc:696-839
//   ORBmatcher::SearchForInitialization                  ORBmatcher.cc:539-683
//
// k_bow: the reference walks the shared vocabulary nodes in ascending order and, inside
// a node, its side-1 features in list order, each taking the best unclaimed side-2
// feature of the same node.  A side-2 feature belongs to exactly one node, so claims
// never cross nodes: nodes are independent and run one per wave, while the features of
// a node run in order inside the wave (lanes = the node's side-2 candidates), which is
// the reference's claim sequence exactly.
//
// k_init: candidates come from a grid window and windows overlap, and a later F1
// keypoint may take an F2 keypoint from an earlier one when its distance is strictly
// smaller (vMatchedDistance).  That distance only ever decreases, so a candidate that
// is unavailable stays unavailable.  All 16 waves first list each query's 8 nearest
// window candidates in (distance, iteration order); wave 0 then replays the queries in
// order, taking the first two still-available entries of each list, and rescans the
// window only when a truncated list runs out.
#include <hip/hip_runtime.h>

#include <climits>

#include "orbx_gmem.h"
#include "orbx_kernels.h"

namespace orbx {

// Orders a wave's LDS accesses between the steps of a single-wave sequential loop (a
// wave's LDS operations execute in issue order, so this only stops the compiler from
// moving them).  Unlike a workgroup fence it does not wait for the wave's outstanding
// global stores, which would put a memory round trip into every step.
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

namespace {

constexpr int kBowThreads = 1024;
constexpr int kBowWaves = kBowThreads / 64;
constexpr int kThLow = 50;          // ORBmatcher::TH_LOW, ORBmatcher.cc:39
constexpr int kInitList = 8;        // listed candidates per initialisation query
constexpr unsigned long long kNone = ~0ull;

// v of lane `src` (wave-uniform src) in every lane
__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int src) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, src);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), src);
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
    const int lo = __shfl_xor((int)(unsigned)v, o, 64), hi = __shfl_xor((int)(unsigned)(v >> 32), o, 64);
    return (unsigned long long)(unsigned)hi << 32 | (unsigned)lo;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = shfl_xor_u64(v, o);
        v = w < v ? w : v;
    }
    return v;
}

__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned w = (unsigned)__shfl_xor((int)v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

struct Desc {
    unsigned long long a, b, c, d;
};

__device__ __forceinline__ Desc load_desc(const uint8_t* p) {
    const ulonglong2* q = (const ulonglong2*)p;
    const ulonglong2 a = ldg(q), b = ldg(q + 1);
    return Desc{a.x, a.y, b.x, b.y};
}

// DescriptorDistance, ORBmatcher.cc:1983-2003
__device__ __forceinline__ int hamming(const Desc& x, const uint8_t* p) {
    const ulonglong2* q = (const ulonglong2*)p;
    const ulonglong2 a = ldg(q), b = ldg(q + 1);
    return __popcll(x.a ^ a.x) + __popcll(x.b ^ a.y) + __popcll(x.c ^ b.x) + __popcll(x.d ^ b.y);
}

// rotHist bin of a match (ORBmatcher.cc:363-371)
__device__ __forceinline__ int rot_bin(float a1, float a2) {
    const float factor = kHistoLength / 360.0f;
    float rot = a1 - a2;
    if (rot < 0.0f) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == kHistoLength) bin = 0;
    return bin;
}

// ComputeThreeMaxima, ORBmatcher.cc:1935-1977, on LDS bin counts (one thread).
__device__ void three_maxima(const int* h, int* ind) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < kHistoLength; i++) {
        const int s = h[i];
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
    if (max2 < 0.1f * (float)max1) {
        ind2 = -1;
        ind3 = -1;
    } else if (max3 < 0.1f * (float)max1) {
        ind3 = -1;
    }
    ind[0] = ind1;
    ind[1] = ind2;
    ind[2] = ind3;
}

}  // namespace

// ------------------------------------------------------------------ SearchByBoW

__global__ __launch_bounds__(kBowThreads) void k_bow(const BowProblem* __restrict__ probs) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_hist[kHistoLength];
    __shared__ int s_ind[3];
    __shared__ int s_nrec;
    const BowProblem pb = probs[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // claimed2: the reference's vpMapPointMatches[idxF] != NULL (KF->F) / vbMatched2 (KF->KF)
    uint8_t* claimed2 = smem;
    int* items = (int*)(smem + ((pb.n2 + 15) & ~15));
    uint8_t* bins = (uint8_t*)(items + (pb.kf_kf ? pb.n1 : pb.n2));
    for (int i = tid; i < pb.n2; i += kBowThreads) claimed2[i] = 0;
    if (tid < kHistoLength) s_hist[tid] = 0;
    if (tid == 0) s_nrec = 0;
    __syncthreads();
    const int acc_th = pb.kf_kf ? kThLow - 1 : kThLow;  // KF->KF: bestDist1 < TH_LOW; KF->F: <= TH_LOW
    for (int nd = wave; nd < pb.nnodes; nd += kBowWaves) {
        const BowNode N = ldg(pb.nodes + nd);
        const int ncand = N.c_end - N.c_beg;
        for (int q = N.q_beg; q < N.q_end; q++) {
            const int idx1 = ldg(pb.q_idx1 + q);
            const Desc d1 = load_desc(pb.desc1 + (size_t)idx1 * 32);
            // lane-local best two of (dist << 16 | node-list position); ties go to the
            // earlier position like the reference's strict '<' updates
            unsigned k1 = 0xffffffffu, k2 = 0xffffffffu;
            for (int p = lane; p < ncand; p += 64) {
                const int idx2 = ldg(pb.fv2_idx + N.c_beg + p);
                if (claimed2[idx2] || (pb.avail2 && !ldg(pb.avail2 + idx2))) continue;
                const int dist = hamming(d1, pb.desc2 + (size_t)idx2 * 32);
                if (dist >= 256) continue;  // never below the initial bestDist 256
                const unsigned key = (unsigned)dist << 16 | (unsigned)p;
                if (key < k1) {
                    k2 = k1;
                    k1 = key;
                } else if (key < k2) {
                    k2 = key;
                }
            }
            const unsigned m1 = wave_min_u32(k1);
            const unsigned m2 = wave_min_u32(k1 == m1 ? k2 : k1);
            const int best1 = m1 == 0xffffffffu ? 256 : (int)(m1 >> 16);
            const int best2 = m2 == 0xffffffffu ? 256 : (int)(m2 >> 16);
            if (best1 <= acc_th && (float)best1 < pb.nnratio * (float)best2) {
                const int idx2 = pb.fv2_idx[N.c_beg + (int)(m1 & 0xffffu)];
                if (lane == 0) {
                    claimed2[idx2] = 1;
                    int item;
                    if (pb.kf_kf) {
                        pb.matches[idx1] = pb.mp2[idx2];
                        item = idx1;
                    } else {
                        pb.matches[idx2] = pb.mp1[idx1];
                        item = idx2;
                    }
                    if (pb.check_ori) {
                        const int bin = rot_bin(pb.keys1[idx1].angle, pb.keys2[idx2].angle);
                        const int r = atomicAdd(&s_nrec, 1);
                        items[r] = item;
                        bins[r] = (uint8_t)bin;
                        atomicAdd(&s_hist[bin], 1);
                    }
                }
                wave_lds_fence();
            }
        }
    }
    if (!pb.check_ori) return;
    __syncthreads();
    if (tid == 0) three_maxima(s_hist, s_ind);
    __syncthreads();
    const int nrec = s_nrec;
    for (int r = tid; r < nrec; r += kBowThreads) {
        const int b = bins[r];
        if (b != s_ind[0] && b != s_ind[1] && b != s_ind[2]) pb.matches[items[r]] = -1;
    }
}

hipError_t launch_bow(const BowProblem* d_prob, int n2, int nitems, hipStream_t stream) {
    const size_t lds = (size_t)((n2 + 15) & ~15) + (size_t)nitems * 5 + 16;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)k_bow, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_bow, dim3(1), dim3(kBowThreads), lds, stream, d_prob);
    return hipGetLastError();
}

// ------------------------------------------------------------------ SearchForInitialization

namespace {

// Window of query q (Frame::GetFeaturesInArea(x, y, windowSize, 0, 0), Frame.cc:488-548):
// cells ix x [y0, y1]; the cells of one grid column are contiguous in the CSR, so
// column ix's candidates are cell_idx[cell_start[ix*ROWS + y0] .. cell_start[ix*ROWS + y1 + 1]).
struct Window {
    int x0, x1, y0, y1;
    bool empty;
};

__device__ __forceinline__ Window init_window(const InitProblem& pb, float x, float y) {
    Window w;
    int t = (int)floorf((x - pb.min_x - pb.r) * pb.inv_w);
    w.x0 = t > 0 ? t : 0;
    t = (int)ceilf((x - pb.min_x + pb.r) * pb.inv_w);
    w.x1 = t < kGridCols - 1 ? t : kGridCols - 1;
    t = (int)floorf((y - pb.min_y - pb.r) * pb.inv_h);
    w.y0 = t > 0 ? t : 0;
    t = (int)ceilf((y - pb.min_y + pb.r) * pb.inv_h);
    w.y1 = t < kGridRows - 1 ? t : kGridRows - 1;
    w.empty = w.x0 >= kGridCols || w.x1 < 0 || w.y0 >= kGridRows || w.y1 < 0;
    return w;
}

// Candidate entry: dist << 40 | iteration rank << 20 | F2 index (ranks and indices < 2^20).
__device__ __forceinline__ int e_dist(unsigned long long e) { return (int)(e >> 40); }
__device__ __forceinline__ int e_idx(unsigned long long e) { return (int)(e & 0xfffffu); }

// Walk query q's window; every lane keeps its best `K` entries in ascending order and
// counts the candidates it saw.  md: vMatchedDistance filter (rescans) or null.
template <int K>
__device__ void init_scan(const InitProblem& pb, int i1, const int* md, unsigned long long (&l)[K], int& seen) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < K; k++) l[k] = kNone;
    seen = 0;
    const float x = ldg(pb.prev + 2 * i1), y = ldg(pb.prev + 2 * i1 + 1);
    const Window w = init_window(pb, x, y);
    if (w.empty) return;
    const Desc d1 = load_desc(pb.desc1 + (size_t)i1 * 32);
    int rank0 = 0;
    for (int ix = w.x0; ix <= w.x1; ix++) {
        const int a = ldg(pb.cell_start + ix * kGridRows + w.y0), b = ldg(pb.cell_start + ix * kGridRows + w.y1 + 1);
        for (int p = a + lane; p < b; p += 64) {
            const int i2 = ldg(pb.cell_idx + p);
            const orbx_keypoint kp = ldg(pb.keys2 + i2);
            if (kp.octave != 0) continue;  // minLevel = maxLevel = level1 = 0
            const float distx = kp.x - x, disty = kp.y - y;
            if (!(fabsf(distx) < pb.r && fabsf(disty) < pb.r)) continue;
            const int dist = hamming(d1, pb.desc2 + (size_t)i2 * 32);
            if (md && md[i2] <= dist) continue;
            seen++;
            unsigned long long e = (unsigned long long)dist << 40 | (unsigned long long)(rank0 + p - a) << 20 |
                                   (unsigned long long)i2;
#pragma unroll
            for (int k = 0; k < K; k++) {  // sorted insertion
                const unsigned long long lo = e < l[k] ? e : l[k];
                e = e < l[k] ? l[k] : e;
                l[k] = lo;
            }
        }
        rank0 += b - a;
    }
}

}  // namespace

// Phase 1 on its own launch, one wave per query over as many CUs as there are queries
// (a query's window walk is a chain of dependent gathers): each query's 8 nearest window
// candidates into pb.lists, exact up to where a lane holding more than 4 candidates runs
// out (then marked truncated in pb.trunc).
constexpr int kInitScanThreads = 256;

__global__ __launch_bounds__(kInitScanThreads) void k_init_scan(const InitProblem* __restrict__ probs) {
    const InitProblem& pb = probs[0];
    const int lane = threadIdx.x & 63;
    const int q = blockIdx.x * (kInitScanThreads / 64) + (threadIdx.x >> 6);
    if (q >= pb.nq) return;  // whole wave
    unsigned long long l[4];
    int seen;
    init_scan<4>(pb, pb.q_idx1[q], nullptr, l, seen);
    int cnt = 0, tr = 0, used = 0;
    for (; cnt < kInitList; cnt++) {
        const unsigned long long m = wave_min_u64(l[0]);
        if (m == kNone) break;
        if (lane == 0) pb.lists[(size_t)q * kInitList + cnt] = m;
        if (l[0] == m) {  // the owner pops its head
            l[0] = l[1];
            l[1] = l[2];
            l[2] = l[3];
            l[3] = kNone;
            used++;
        }
        // an owner that listed all 4 of more than 4 seen: the next entry is unknown
        const int stop = __any(used == 4 && seen > 4 && l[0] == kNone);
        if (stop) {
            tr = 1;
            cnt++;
            break;
        }
    }
    if (cnt == kInitList && __any(l[0] != kNone || (seen > used && used == 4))) tr = 1;
    if (lane == 0) pb.trunc[q] = cnt | tr << 8;
}

__global__ __launch_bounds__(kBowThreads) void k_init(const InitProblem* __restrict__ probs, int lists_lds) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_hist[kHistoLength];
    __shared__ int s_ind[3];
    __shared__ int s_nrec;
    const InitProblem pb = probs[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // LDS: the candidate lists first (8-byte aligned; in the problem's global buffer
    // when they do not fit), then 4-byte arrays, then the bins
    const unsigned long long* lists = pb.lists;  // [nq * kInitList], from k_init_scan
    const int* trunc = pb.trunc;                 // listed count | truncated << 8 [nq]
    (void)lists_lds;
    int* md = (int*)smem;                        // vMatchedDistance [n2]
    int* m21 = md + pb.n2;         // vnMatches21 [n2]
    int* m12 = m21 + pb.n2;        // vnMatches12 [n1]
    int* items = m12 + pb.n1;      // rotHist entries (F1 index) [nq]
    int* qi1 = items + pb.nq;      // the queries' F1 keypoints [nq]
    float* ang1 = (float*)(qi1 + pb.nq);  // keypoint angles of F1 [n1] and F2 [n2]
    float* ang2 = ang1 + pb.n1;
    int* owner = (int*)(ang2 + pb.n2);  // lowest lane of a commit round taking F2 keypoint i [n2]
    uint8_t* bins = (uint8_t*)(owner + pb.n2);
    for (int i = tid; i < pb.n2; i += kBowThreads) {
        md[i] = INT_MAX;
        m21[i] = -1;
        ang2[i] = pb.keys2[i].angle;
        owner[i] = 0x7fffffff;
    }
    for (int i = tid; i < pb.n1; i += kBowThreads) {
        m12[i] = -1;
        ang1[i] = pb.keys1[i].angle;
    }
    for (int i = tid; i < pb.nq; i += kBowThreads) qi1[i] = pb.q_idx1[i];
    if (tid < kHistoLength) s_hist[tid] = 0;
    if (tid == 0) s_nrec = 0;

    // phase 1 (the candidate lists) ran in k_init_scan
    __syncthreads();

    // phase 2: the reference's sequential loop over F1's level-0 keypoints (wave 0), in
    // rounds over chunks of 64 queries.  A query's decision reads vMatchedDistance only at
    // its listed entries (or, when its truncated list runs short, at its whole window), and
    // a commit changes it at one entry (its best).  So every query before the first one
    // whose list holds a keypoint an earlier query of the round takes (an LDS owner map),
    // or that needs the rescan, decides exactly as in the sequential loop and all of them
    // commit at once; the first conflicting query is then decided alone.
    if (wave == 0) {
        auto decide = [&](int q, unsigned long long& best, unsigned long long& second) {
            // the first two listed entries still available, in list order: lane k checks
            // entry k against vMatchedDistance, the two lowest set ballot bits win
            const int t = trunc[q];
            const int cnt = t & 0xff, tr = t >> 8;
            unsigned long long e = kNone;
            bool avail = false;
            if (lane < cnt) {
                e = lists[(size_t)q * kInitList + lane];
                avail = md[e_idx(e)] > e_dist(e);
            }
            const unsigned long long bal = __ballot(avail);
            const int found = __popcll(bal) < 2 ? __popcll(bal) : 2;
            best = kNone;
            second = kNone;
            if (found >= 1) best = shfl_u64(e, __ffsll((long long)bal) - 1);
            if (found >= 2) second = shfl_u64(e, __ffsll((long long)(bal & (bal - 1))) - 1);
            if (found < 2 && tr) {  // the list ran out: rescan the window against vMatchedDistance
                unsigned long long l[2];
                int seen;
                init_scan<2>(pb, qi1[q], md, l, seen);
                best = wave_min_u64(l[0]);
                second = wave_min_u64(l[0] == best ? l[1] : l[0]);
            }
        };
        auto accepted = [&](unsigned long long best, unsigned long long second) {
            const int bestDist = best == kNone ? INT_MAX : e_dist(best);
            const int bestDist2 = second == kNone ? INT_MAX : e_dist(second);
            return bestDist <= kThLow && (float)bestDist < (float)bestDist2 * pb.nnratio;
        };
        // commit of query i1 taking F2 keypoint i2 (one lane per query)
        auto commit = [&](int i1, unsigned long long best, int slot) {
            const int i2 = e_idx(best);
            const int prev = m21[i2];
            if (prev >= 0) m12[prev] = -1;
            m12[i1] = i2;
            m21[i2] = i1;
            md[i2] = e_dist(best);
            if (pb.check_ori) {
                const int bin = rot_bin(ang1[i1], ang2[i2]);
                items[slot] = i1;
                bins[slot] = (uint8_t)bin;
                atomicAdd(&s_hist[bin], 1);
            }
        };
        int nrec = 0;
        for (int q0 = 0; q0 < pb.nq; q0 += 64) {
            const int q = q0 + lane;
            const bool valid = q < pb.nq;
            // this lane's query: its listed entries and whether the list is truncated
            unsigned long long L[kInitList];
            int cnt = 0, tr = 0, i1 = -1;
            if (valid) {
                const int t = trunc[q];
                cnt = t & 0xff;
                tr = t >> 8;
                i1 = qi1[q];
            }
#pragma unroll
            for (int k = 0; k < kInitList; k++) L[k] = (k < cnt) ? lists[(size_t)q * kInitList + k] : kNone;
            int start = 0;
            while (true) {
                const bool act = valid && lane >= start;
                unsigned long long best = kNone, second = kNone;
                bool rescan = false;
                if (act) {
                    int found = 0;
#pragma unroll
                    for (int k = 0; k < kInitList; k++) {
                        if (L[k] != kNone && found < 2 && md[e_idx(L[k])] > e_dist(L[k])) {
                            if (found == 0) best = L[k];
                            else second = L[k];
                            found++;
                        }
                    }
                    rescan = found < 2 && tr;
                }
                const bool acc = act && !rescan && accepted(best, second);
                if (acc) atomicMin(&owner[e_idx(best)], lane);
                bool conf = rescan;
                if (act && !rescan) {
#pragma unroll
                    for (int k = 0; k < kInitList; k++)
                        if (L[k] != kNone && owner[e_idx(L[k])] < lane) conf = true;
                }
                if (acc) owner[e_idx(best)] = 0x7fffffff;
                const unsigned long long cm = __ballot(conf);
                const int f = cm ? __ffsll((long long)cm) - 1 : 64;
                const bool com = acc && lane < f;
                const unsigned long long comm = __ballot(com);
                if (com) commit(i1, best, nrec + __popcll(comm & ((1ull << lane) - 1ull)));
                if (pb.check_ori) nrec += __popcll(comm);
                if (f >= 64) break;
                wave_lds_fence();
                // query q0 + f alone, against every earlier commit
                unsigned long long b1, b2;
                decide(q0 + f, b1, b2);
                if (accepted(b1, b2)) {
                    if (lane == 0) commit(qi1[q0 + f], b1, nrec);
                    if (pb.check_ori) nrec++;
                }
                start = f + 1;
                wave_lds_fence();
            }
            wave_lds_fence();
        }
        if (lane == 0) s_nrec = nrec;
        wave_lds_fence();
        if (pb.check_ori && lane == 0) three_maxima(s_hist, s_ind);
    }
    __syncthreads();
    if (pb.check_ori) {
        const int nrec = s_nrec;
        for (int r = tid; r < nrec; r += kBowThreads) {
            const int b = bins[r];
            if (b != s_ind[0] && b != s_ind[1] && b != s_ind[2]) m12[items[r]] = -1;
        }
        __syncthreads();
    }
    for (int i = tid; i < pb.n1; i += kBowThreads) pb.matches12[i] = m12[i];
}

hipError_t launch_init(const InitProblem* d_prob, int n1, int n2, int nq, hipStream_t stream) {
    const size_t lds = (size_t)4 * (4 * n2 + 2 * n1 + 2 * nq) + (size_t)nq + 16;
    const int lists_lds = 0;
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    if (nq > 0) {
        const int per = kInitScanThreads / 64;
        hipLaunchKernelGGL(k_init_scan, dim3((nq + per - 1) / per), dim3(kInitScanThreads), 0, stream, d_prob);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)k_init, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_init, dim3(1), dim3(kBowThreads), lds, stream, d_prob, lists_lds);
    return hipGetLastError();
}

}  // namespace orbx
