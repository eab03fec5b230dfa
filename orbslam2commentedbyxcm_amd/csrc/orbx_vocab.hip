// orbx_vocab.hip -- DBoW2 vocabulary transform (TemplatedVocabulary<FORB::TDescriptor,
// FORB>, Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h) for gfx950, behind include/orbx.h.
//
// Device layout.  The tree is stored as its edge list in CSR order:
// the children of node p occupy edge slots [off(p), off(p) + cnt(p)) in file order, so
// one node's k child descriptors are one contiguous 32*k-byte run.  Per edge slot:
//   edesc  2 x uint4   the child's 256-bit descriptor
//   einfo  int4        (off, cnt) of the child's own children (cnt == 0 -> leaf), the
//                      child's node id and word id
//   eweight double     the child's weight
// ORBvoc.txt (k=10, L=6, ~1.1M nodes) is ~62 MB in this form: the upper levels stay in
// L2, the rest in the Infinity Cache.
//
// k_vocab_walk: one 16-lane row per descriptor (four per wave), one lane per child.
//   Each level is a 16-wide Hamming + DPP row minimum of (distance << 16 | child),
//   so ties resolve to the first child in file order like the reference's strict '<'.
//   Every lane loads its child's einfo together with the descriptor and the winner's
//   is taken by lane shuffle, so a level costs one dependent global load, not two.
// k_vocab_frame: one workgroup per frame builds the BowVector (word -> value map,
//   BowVector.cpp) and FeatureVector (node -> ascending feature indices,
//   FeatureVector.cpp:31-45) from the per-feature words: LDS bitonic sort of
//   (id << 32 | feature) keys, run heads, a sequential double sum per run in feature
//   order (addWeight) and a sequential norm in ascending word order (normalize), so
//   every double is bit-identical to the reference's std::map walk.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "orbx.h"
#include "orbx_block_sort.h"
#include "orbx_error.h"

using namespace orbx;

namespace orbx {
namespace {

constexpr int kVocMaxCap = 8192;   // features per frame in one transform (LDS sort size)
constexpr int kFrameThreads = 1024;
constexpr int kWalkThreads = 256;  // 16 descriptors per block
static_assert(kFrameThreads == kSortThreads && kVocMaxCap == kSortMaxKeys, "orbx_block_sort.h geometry");

__device__ __forceinline__ unsigned umin_(unsigned a, unsigned b) { return a < b ? a : b; }

}  // namespace

// Minimum over each 16-lane DPP row, broadcast to the row (quad_perm x2, half mirror,
// mirror).
__device__ __forceinline__ unsigned row_min16(unsigned v) {
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false));
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false));
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false));
    v = umin_(v, (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false));
    return v;
}

struct VocDev {
    const uint4* edesc;
    const int4* einfo;
    const double* eweight;
    int root_cnt;
    int max_depth;
};

// TemplatedVocabulary::transform(feature, word_id, weight, nid, levelsup),
// TemplatedVocabulary.h:1220-1259.  Frame b's descriptors at desc + (b*cap + i)*32,
// i < n[b].  Outputs per feature slot: word, weight, node at level L - levelsup.
__global__ __launch_bounds__(kWalkThreads) void k_vocab_walk(VocDev V, const uint8_t* __restrict__ desc,
                                                            const int32_t* __restrict__ nper, int cap,
                                                            int nid_level, int32_t* __restrict__ feat_word,
                                                            double* __restrict__ feat_weight,
                                                            int32_t* __restrict__ feat_node) {
    const int b = blockIdx.y;
    const int n = min(nper[b], cap);
    const int i = blockIdx.x * (kWalkThreads / 16) + (threadIdx.x >> 4);
    const int sub = threadIdx.x & 15;
    if (blockIdx.x * (kWalkThreads / 16) >= n) return;  // whole block past the frame's count
    const bool live = i < n;
    const size_t slot = (size_t)b * cap + (live ? i : 0);
    const uint4* q = (const uint4*)(desc + slot * 32);
    const uint4 q0 = q[0], q1 = q[1];
    int off = 0, cnt = V.root_cnt, node = 0, nid = 0, word = 0, e = -1;
    const int rowbase = threadIdx.x & ~15;
    // Each row leaves at its leaf; off/cnt are row-uniform, so a row's 16 lanes stay
    // converged for the DPP minimum and the shuffles.  max_depth bounds the walk.
    for (int level = 1; level <= V.max_depth && cnt > 0; level++) {
        unsigned best = 0xffffffffu;
        int4 mine = make_int4(0, 0, 0, 0);  // einfo of this lane's best child
        for (int c0 = 0; c0 < cnt; c0 += 16) {
            const int j = c0 + sub;
            if (j < cnt) {
                const uint4* ed = V.edesc + 2 * (size_t)(off + j);
                const uint4 a = ed[0], c = ed[1];
                const int4 inf = V.einfo[off + j];
                const unsigned d = __popc(a.x ^ q0.x) + __popc(a.y ^ q0.y) + __popc(a.z ^ q0.z) +
                                   __popc(a.w ^ q0.w) + __popc(c.x ^ q1.x) + __popc(c.y ^ q1.y) +
                                   __popc(c.z ^ q1.z) + __popc(c.w ^ q1.w);
                const unsigned key = d << 16 | (unsigned)j;
                if (key < best) {
                    best = key;
                    mine = inf;
                }
            }
        }
        best = row_min16(best);
        const int src = rowbase | (int)(best & 15u);  // the lane that scored the winner
        e = off + (int)(best & 0xffffu);
        off = __shfl(mine.x, src, 64);
        cnt = __shfl(mine.y, src, 64);
        node = __shfl(mine.z, src, 64);
        word = __shfl(mine.w, src, 64);
        if (level <= nid_level) nid = node;  // leaf above nid_level: deepest node
    }
    if (live && sub == 0) {
        feat_word[slot] = word;
        feat_weight[slot] = e >= 0 ? V.eweight[e] : 0.0;
        if (feat_node) feat_node[slot] = nid_level <= 0 ? 0 : nid;
    }
}

// Exclusive block scan of one int per thread (kFrameThreads), returns the total.
__device__ int block_scan(int v, int* s_wave, int& excl) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[wv] = x;
    __syncthreads();
    if (threadIdx.x < 64) {
        int w = threadIdx.x < kFrameThreads / 64 ? s_wave[threadIdx.x] : 0;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(w, o, 64);
            if ((int)threadIdx.x >= o) w += y;
        }
        if (threadIdx.x < kFrameThreads / 64) s_wave[16 + threadIdx.x] = w;  // inclusive over waves
    }
    __syncthreads();
    excl = x - v + (wv ? s_wave[16 + wv - 1] : 0);
    const int total = s_wave[16 + kFrameThreads / 64 - 1];
    __syncthreads();
    return total;
}

// Run heads of the sorted keys s[0, nw): each thread owns `per` consecutive entries.
// Writes head positions via `emit(pos, i)`; returns the number of runs.
template <typename Emit>
__device__ int scan_heads(const unsigned long long* s, int nw, int per, int* s_wave, Emit emit) {
    const int lo = threadIdx.x * per;
    int cnt = 0;
    for (int i = lo; i < lo + per && i < nw; i++) cnt += (i == 0 || (s[i] >> 32) != (s[i - 1] >> 32));
    int excl;
    const int total = block_scan(cnt, s_wave, excl);
    for (int i = lo; i < lo + per && i < nw; i++)
        if (i == 0 || (s[i] >> 32) != (s[i - 1] >> 32)) emit(excl++, i);
    return total;
}

struct FrameOut {
    int32_t* bow_word;
    double* bow_value;
    int32_t* nbow;
    int32_t* fv_node;
    int32_t* fv_off;
    int32_t* fv_idx;
    int32_t* nfv;
};

// TemplatedVocabulary::transform(features, BowVector&, FeatureVector&, levelsup),
// TemplatedVocabulary.h:1127-1186; BowVector::addWeight / addIfNotExist / normalize
// (BowVector.cpp:34-84); FeatureVector::addFeature (FeatureVector.cpp:31-45).
// accumulate: TF / TF_IDF; norm: 0 none, 1 L1, 2 L2 (ScoringObject.h mustNormalize).
__global__ __launch_bounds__(kFrameThreads) void k_vocab_frame(const int32_t* __restrict__ nper, int cap,
                                                              const int32_t* __restrict__ feat_word,
                                                              const double* __restrict__ feat_weight,
                                                              const int32_t* __restrict__ feat_node, int np,
                                                              int accumulate, int norm_kind, FrameOut O) {
    extern __shared__ unsigned long long s_key[];  // np keys, then np doubles
    double* s_val = (double*)(s_key + np);
    __shared__ int s_wave[32];
    __shared__ int s_nw;
    __shared__ double s_norm;
    const int b = blockIdx.x;
    const int n = min(nper[b], cap);
    const size_t base = (size_t)b * cap;
    // this frame's sort size: the next power of two >= n, at least 1024 (one key per thread)
    int ne = 1;
    while (ne * kFrameThreads < n) ne <<= 1;
    const int m = ne * kFrameThreads;
    const int per = ne;
    unsigned long long r[kSortPer];

    // ---- BowVector: sort (word, feature) over non-stopped features
#pragma unroll
    for (int e = 0; e < kSortPer; e++) {
        const int i = e * kFrameThreads + threadIdx.x;
        r[e] = (e < ne && i < n && feat_weight[base + i] > 0)
                   ? ((unsigned long long)(unsigned)feat_word[base + i] << 32 | (unsigned)i)
                   : ~0ull;
    }
    if (threadIdx.x == 0) s_nw = 0;
    block_bitonic_sort64(r, ne, s_key);
    for (int i = threadIdx.x; i < m; i += kFrameThreads)
        if (s_key[i] != ~0ull && (i + 1 == m || s_key[i + 1] == ~0ull)) s_nw = i + 1;
    __syncthreads();
    const int nw = s_nw;
    // s_val[p] = value of run p; runs summed in feature order (addWeight) or first (addIfNotExist)
    const int nb = scan_heads(s_key, nw, per, s_wave, [&](int p, int i) {
        const unsigned w = (unsigned)(s_key[i] >> 32);
        double v = feat_weight[base + (unsigned)s_key[i]];
        if (accumulate)
            for (int j = i + 1; j < nw && (unsigned)(s_key[j] >> 32) == w; j++)
                v = __dadd_rn(v, feat_weight[base + (unsigned)s_key[j]]);
        s_val[p] = v;
        O.bow_word[base + p] = (int32_t)w;
    });
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        if (norm_kind == 1) {
            for (int p = 0; p < nb; p++) s = __dadd_rn(s, fabs(s_val[p]));
        } else if (norm_kind == 2) {
            // fused like the reference's build (g++ -O3 -march=native contracts C++:
            // BowVector::normalize's L2 loop is one vfmadd; tests/test_vocab_ref.py)
            for (int p = 0; p < nb; p++) s = __fma_rn(s_val[p], s_val[p], s);
            s = sqrt(s);
        } else {
            s = accumulate ? (double)nb : 0.0;  // TF / TF_IDF without normalisation: / size()
        }
        s_norm = s;
        O.nbow[b] = nb;
    }
    __syncthreads();
    const double s = s_norm;
    for (int p = threadIdx.x; p < nb; p += kFrameThreads)
        O.bow_value[base + p] = (s > 0.0) ? s_val[p] / s : s_val[p];
    __syncthreads();

    // ---- FeatureVector: sort (node, feature) over the same features
#pragma unroll
    for (int e = 0; e < kSortPer; e++) {
        const int i = e * kFrameThreads + threadIdx.x;
        r[e] = (e < ne && i < n && feat_weight[base + i] > 0)
                   ? ((unsigned long long)(unsigned)feat_node[base + i] << 32 | (unsigned)i)
                   : ~0ull;
    }
    block_bitonic_sort64(r, ne, s_key);
    for (int i = threadIdx.x; i < nw; i += kFrameThreads) O.fv_idx[base + i] = (int32_t)(unsigned)s_key[i];
    const int nf = scan_heads(s_key, nw, per, s_wave, [&](int p, int i) {
        O.fv_node[base + p] = (int32_t)(s_key[i] >> 32);
        O.fv_off[b * (size_t)(cap + 1) + p] = i;
    });
    if (threadIdx.x == 0) {
        O.fv_off[b * (size_t)(cap + 1) + nf] = nw;
        O.nfv[b] = nf;
    }
}

}  // namespace orbx

// ---------------------------------------------------------------------------------------
// Host side

struct orbx_vocabulary {
    int device = 0;
    int k = 0, L = 0, scoring = 0, weighting = 0;
    int nnodes = 0, nwords = 0, max_depth = 0, root_cnt = 0;
    hipStream_t stream = nullptr;
    uint4* edesc = nullptr;
    int4* einfo = nullptr;
    double* eweight = nullptr;
    // grow-only work buffers: per-feature words/weights/nodes, host-API staging
    char* work = nullptr;
    size_t work_cap = 0;
    static constexpr int kRing = 64;
    bool timing = false;
    hipEvent_t ev[kRing][3] = {};
    long long ncalls = 0;
};

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

struct HostTree {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    std::vector<uint8_t> desc;  // node-major, 32 B
    std::vector<int> parent, word;
    std::vector<double> weight;
};

bool parse_long(const char*& p, const char* end, long& out) {
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\r')) p++;
    if (p >= end) return false;
    char* e = nullptr;
    errno = 0;
    out = std::strtol(p, &e, 10);
    if (e == p || errno) return false;
    p = e;
    return true;
}

// loadFromTextFile, TemplatedVocabulary.h:1338-1424 (the text is NUL-terminated by the
// caller so strtol/strtod never read past it).  Empty lines are skipped; the
// reference turns each into a bogus root child with an uninitialised descriptor
// (DESIGN.md §4.8).  Malformed node lines are an error here.
int parse_text(const char* text, size_t len, HostTree& t) {
    const char* p = text;
    const char* end = text + len;
    const char* nl = (const char*)memchr(p, '\n', (size_t)(end - p));
    const char* le = nl ? nl : end;
    long h[4];
    const char* q = p;
    for (int i = 0; i < 4; i++)
        if (!parse_long(q, le, h[i])) return fail(ORBX_ERR_ARG, "vocabulary header: expected 'k L scoring weighting'");
    if (h[0] < 0 || h[0] > 20 || h[1] < 1 || h[1] > 10 || h[2] < 0 || h[2] > 5 || h[3] < 0 || h[3] > 3)
        return fail(ORBX_ERR_ARG, "Vocabulary loading failure: This is not a correct text file!");
    t.k = (int)h[0];
    t.L = (int)h[1];
    t.scoring = (int)h[2];
    t.weighting = (int)h[3];
    t.desc.assign(32, 0);
    t.parent.assign(1, 0);
    t.word.assign(1, 0);
    t.weight.assign(1, 0.0);
    int nwords = 0;
    p = nl ? nl + 1 : end;
    while (p < end) {
        nl = (const char*)memchr(p, '\n', (size_t)(end - p));
        le = nl ? nl : end;
        const char* s = p;
        p = nl ? nl + 1 : end;
        while (s < le && (*s == ' ' || *s == '\t' || *s == '\r')) s++;
        if (s == le) continue;
        const int nid = (int)t.parent.size();
        long pid, leaf, v;
        if (!parse_long(s, le, pid) || !parse_long(s, le, leaf)) return fail(ORBX_ERR_ARG, "vocabulary node line");
        if (pid < 0 || pid >= nid) return fail(ORBX_ERR_ARG, "vocabulary node: parent id out of range");
        uint8_t d[32];
        for (int i = 0; i < 32; i++) {
            if (!parse_long(s, le, v)) return fail(ORBX_ERR_ARG, "vocabulary node: descriptor");
            d[i] = (uint8_t)v;  // FORB::fromString: (unsigned char)n
        }
        while (s < le && (*s == ' ' || *s == '\t')) s++;
        char* e = nullptr;
        const double w = std::strtod(s, &e);
        if (e == s || e > le) return fail(ORBX_ERR_ARG, "vocabulary node: weight");
        t.desc.insert(t.desc.end(), d, d + 32);
        t.parent.push_back((int)pid);
        t.word.push_back(leaf > 0 ? nwords++ : 0);  // Node() default word_id 0
        t.weight.push_back(w);
        if (t.parent.size() > (size_t)0x7fffffff / 2) return fail(ORBX_ERR_ARG, "vocabulary too large");
    }
    return ORBX_OK;
}

int upload(orbx_vocabulary* v, const HostTree& t) {
    const int n = (int)t.parent.size();
    const int E = n - 1;
    std::vector<int> off(n + 1, 0), depth(n, 0);
    for (int i = 1; i < n; i++) off[t.parent[i] + 1]++;
    for (int i = 0; i < n; i++) {
        if (off[i + 1] > 65535) return fail(ORBX_ERR_UNSUPPORTED, "vocabulary node with more than 65535 children");
        off[i + 1] += off[i];
    }
    std::vector<int> fill(off.begin(), off.end() - 1);
    std::vector<uint8_t> edesc((size_t)(E > 0 ? E : 1) * 32);
    std::vector<int4> einfo(E > 0 ? E : 1);
    std::vector<double> eweight(E > 0 ? E : 1);
    int max_depth = 0;
    for (int i = 1; i < n; i++) {
        const int e = fill[t.parent[i]]++;
        std::memcpy(&edesc[(size_t)e * 32], &t.desc[(size_t)i * 32], 32);
        einfo[e] = make_int4(off[i], off[i + 1] - off[i], i, t.word[i]);
        eweight[e] = t.weight[i];
        depth[i] = depth[t.parent[i]] + 1;
        if (depth[i] > max_depth) max_depth = depth[i];
    }
    v->k = t.k;
    v->L = t.L;
    v->scoring = t.scoring;
    v->weighting = t.weighting;
    v->nnodes = n;
    v->root_cnt = off[1] - off[0];
    v->max_depth = max_depth;
    HIP_TRY(hipMalloc((void**)&v->edesc, edesc.size()));
    HIP_TRY(hipMalloc((void**)&v->einfo, sizeof(int4) * einfo.size()));
    HIP_TRY(hipMalloc((void**)&v->eweight, sizeof(double) * eweight.size()));
    HIP_TRY(hipMemcpy(v->edesc, edesc.data(), edesc.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(v->einfo, einfo.data(), sizeof(int4) * einfo.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(v->eweight, eweight.data(), sizeof(double) * eweight.size(), hipMemcpyHostToDevice));
    return ORBX_OK;
}

void free_vocab(orbx_vocabulary* v) {
    void* ptrs[] = {v->edesc, v->einfo, v->eweight, v->work};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (auto& slot : v->ev)
        for (auto& e : slot)
            if (e) (void)hipEventDestroy(e);
    if (v->stream) (void)hipStreamDestroy(v->stream);
}

int reserve_work(orbx_vocabulary* v, size_t bytes) {
    if (bytes <= v->work_cap) return ORBX_OK;
    if (v->work) (void)hipFree(v->work);
    v->work = nullptr;
    v->work_cap = 0;
    HIP_TRY(hipMalloc((void**)&v->work, bytes));
    v->work_cap = bytes;
    return ORBX_OK;
}

size_t up256(size_t b) { return (b + 255) & ~(size_t)255; }

int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

// ScoringObject::mustNormalize (ScoringObject.h:74-89 per class): L1 for L1 / ChiSquare
// / KL / Bhattacharyya, L2 for L2, none for DotProduct.
int norm_kind(int scoring) { return scoring == 1 ? 2 : (scoring == 5 ? 0 : 1); }

int launch(orbx_vocabulary* v, int batch, const uint8_t* d_desc, const int32_t* d_n, int cap, int levelsup,
           int32_t* feat_word, double* feat_weight, int32_t* feat_node, const FrameOut& O, hipStream_t s,
           bool need_frame) {
    VocDev V{v->edesc, v->einfo, v->eweight, v->root_cnt, v->max_depth};
    hipEvent_t* ev = nullptr;
    if (v->timing) {
        ev = v->ev[v->ncalls % orbx_vocabulary::kRing];
        for (int i = 0; i < 3; i++)
            if (!ev[i]) HIP_TRY(hipEventCreate(&ev[i]));
        HIP_TRY(hipEventRecord(ev[0], s));
    }
    const dim3 g1((cap + kWalkThreads / 16 - 1) / (kWalkThreads / 16), batch);
    k_vocab_walk<<<g1, kWalkThreads, 0, s>>>(V, d_desc, d_n, cap, v->L - levelsup, feat_word, feat_weight,
                                             feat_node);
    HIP_TRY(hipGetLastError());
    if (ev) HIP_TRY(hipEventRecord(ev[1], s));
    if (need_frame) {
        const int np = next_pow2(cap < kFrameThreads ? kFrameThreads : cap);
        const size_t lds = (size_t)np * 16;
        static thread_local bool attr = false;
        if (!attr) {
            HIP_TRY(hipFuncSetAttribute((const void*)k_vocab_frame, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)((size_t)kVocMaxCap * 16)));
            attr = true;
        }
        k_vocab_frame<<<batch, kFrameThreads, lds, s>>>(d_n, cap, feat_word, feat_weight, feat_node, np,
                                                       v->weighting == 0 || v->weighting == 1,
                                                       norm_kind(v->scoring), O);
        HIP_TRY(hipGetLastError());
    }
    if (ev) {
        HIP_TRY(hipEventRecord(ev[2], s));
        v->ncalls++;
    }
    return ORBX_OK;
}

}  // namespace

extern "C" {

int orbx_vocabulary_load_text(const char* text, size_t len, int device, orbx_vocabulary** out) {
    if (!out || (!text && len)) return fail(ORBX_ERR_ARG, "null argument");
    *out = nullptr;
    std::string buf(text ? text : "", len);  // NUL-terminated copy for strtol/strtod
    HostTree t;
    int rc = parse_text(buf.c_str(), buf.size(), t);
    if (rc != ORBX_OK) return rc;
    orbx_vocabulary* v = new (std::nothrow) orbx_vocabulary();
    if (!v) return fail(ORBX_ERR_ARG, "out of host memory");
    v->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        free_vocab(v);
        delete v;
        set_last_error(std::string("orbx_vocabulary_load_text: ") + hipGetErrorString(e));
        return ORBX_ERR_HIP;
    }
    rc = upload(v, t);
    if (rc != ORBX_OK) {
        free_vocab(v);
        delete v;
        return rc;
    }
    int nw = 0;
    for (size_t i = 1; i < t.word.size(); i++)
        if (t.word[i] + 1 > nw) nw = t.word[i] + 1;
    v->nwords = nw;
    *out = v;
    return ORBX_OK;
}

int orbx_vocabulary_load_text_file(const char* path, int device, orbx_vocabulary** out) {
    if (!out || !path) return fail(ORBX_ERR_ARG, "null argument");
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(ORBX_ERR_ARG, "cannot open vocabulary file");
    std::string buf;
    char chunk[1 << 16];
    size_t r;
    while ((r = std::fread(chunk, 1, sizeof(chunk), f)) > 0) buf.append(chunk, r);
    std::fclose(f);
    return orbx_vocabulary_load_text(buf.data(), buf.size(), device, out);
}

void orbx_vocabulary_destroy(orbx_vocabulary* v) {
    if (!v || orbx::unloading()) return;
    (void)hipSetDevice(v->device);
    if (v->stream) (void)hipStreamSynchronize(v->stream);
    free_vocab(v);
    delete v;
}

int orbx_vocabulary_info(const orbx_vocabulary* v, int* k, int* L, int* scoring, int* weighting, int* nnodes,
                         int* nwords) {
    if (!v) return fail(ORBX_ERR_ARG, "null vocabulary");
    if (k) *k = v->k;
    if (L) *L = v->L;
    if (scoring) *scoring = v->scoring;
    if (weighting) *weighting = v->weighting;
    if (nnodes) *nnodes = v->nnodes;
    if (nwords) *nwords = v->nwords;
    return ORBX_OK;
}

void* orbx_vocabulary_stream(orbx_vocabulary* v) { return v ? (void*)v->stream : nullptr; }

int orbx_vocabulary_transform_features(orbx_vocabulary* v, const uint8_t* desc, int n, int levelsup, int32_t* word,
                                       double* weight, int32_t* node) {
    if (!v || n < 0 || (n && (!desc || !word || !weight))) return fail(ORBX_ERR_ARG, "null argument");
    if (n == 0) return ORBX_OK;
    if (v->nwords == 0) return fail(ORBX_ERR_STATE, "empty vocabulary");
    HIP_TRY(hipSetDevice(v->device));
    const size_t b_desc = up256((size_t)n * 32), b_i = up256((size_t)n * 4), b_d = up256((size_t)n * 8);
    int rc = reserve_work(v, b_desc + 3 * b_i + b_d + 256);
    if (rc) return rc;
    uint8_t* d_desc = (uint8_t*)v->work;
    int32_t* d_word = (int32_t*)(v->work + b_desc);
    int32_t* d_node = (int32_t*)(v->work + b_desc + b_i);
    int32_t* d_n = (int32_t*)(v->work + b_desc + 2 * b_i);
    double* d_weight = (double*)(v->work + b_desc + 3 * b_i);
    HIP_TRY(hipMemcpyAsync(d_desc, desc, (size_t)n * 32, hipMemcpyHostToDevice, v->stream));
    HIP_TRY(hipMemcpyAsync(d_n, &n, 4, hipMemcpyHostToDevice, v->stream));
    rc = launch(v, 1, d_desc, d_n, n, levelsup, d_word, d_weight, d_node, FrameOut{}, v->stream, false);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(word, d_word, (size_t)n * 4, hipMemcpyDeviceToHost, v->stream));
    HIP_TRY(hipMemcpyAsync(weight, d_weight, (size_t)n * 8, hipMemcpyDeviceToHost, v->stream));
    if (node) HIP_TRY(hipMemcpyAsync(node, d_node, (size_t)n * 4, hipMemcpyDeviceToHost, v->stream));
    HIP_TRY(hipStreamSynchronize(v->stream));
    return ORBX_OK;
}

int orbx_vocabulary_transform_batch_device(orbx_vocabulary* v, int batch, const uint8_t* d_desc, const int32_t* d_n,
                                           int cap, int levelsup, int32_t* d_feat_word, int32_t* d_feat_node,
                                           int32_t* d_bow_word, double* d_bow_value, int32_t* d_nbow,
                                           int32_t* d_fv_node, int32_t* d_fv_off, int32_t* d_fv_idx, int32_t* d_nfv,
                                           void* stream) {
    if (!v || batch < 0 || cap < 0) return fail(ORBX_ERR_ARG, "bad argument");
    if (batch == 0 || cap == 0) return ORBX_OK;
    if (!d_desc || !d_n || !d_bow_word || !d_bow_value || !d_nbow || !d_fv_node || !d_fv_off || !d_fv_idx || !d_nfv)
        return fail(ORBX_ERR_ARG, "null argument");
    if (cap > kVocMaxCap) return fail(ORBX_ERR_UNSUPPORTED, "more than 8192 features per frame");
    HIP_TRY(hipSetDevice(v->device));
    hipStream_t s = stream ? (hipStream_t)stream : v->stream;
    if (v->nwords == 0) {  // transform() on an empty vocabulary: empty vectors
        HIP_TRY(hipMemsetAsync(d_nbow, 0, sizeof(int32_t) * (size_t)batch, s));
        HIP_TRY(hipMemsetAsync(d_nfv, 0, sizeof(int32_t) * (size_t)batch, s));
        HIP_TRY(hipMemsetAsync(d_fv_off, 0, sizeof(int32_t) * (size_t)batch * (cap + 1), s));
        return ORBX_OK;
    }
    const size_t slots = (size_t)batch * cap;
    const size_t b_i = up256(slots * 4), b_d = up256(slots * 8);
    const size_t need = (d_feat_word ? 0 : b_i) + (d_feat_node ? 0 : b_i) + b_d + 256;
    int rc = reserve_work(v, need);
    if (rc) return rc;
    char* w = v->work;
    double* feat_weight = (double*)w;
    w += b_d;
    if (!d_feat_word) {
        d_feat_word = (int32_t*)w;
        w += b_i;
    }
    if (!d_feat_node) d_feat_node = (int32_t*)w;
    return launch(v, batch, d_desc, d_n, cap, levelsup, d_feat_word, feat_weight, d_feat_node,
                  FrameOut{d_bow_word, d_bow_value, d_nbow, d_fv_node, d_fv_off, d_fv_idx, d_nfv}, s, true);
}

int orbx_vocabulary_transform(orbx_vocabulary* v, const uint8_t* desc, int n, int levelsup, int32_t* bow_word,
                              double* bow_value, int* nbow, int32_t* fv_node, int32_t* fv_off, int32_t* fv_idx,
                              int* nfv) {
    if (!v || n < 0 || !nbow || !nfv || !fv_off || (n && (!desc || !bow_word || !bow_value || !fv_node || !fv_idx)))
        return fail(ORBX_ERR_ARG, "null argument");
    *nbow = 0;
    *nfv = 0;
    fv_off[0] = 0;
    if (n == 0 || v->nwords == 0) return ORBX_OK;
    if (n > kVocMaxCap) return fail(ORBX_ERR_UNSUPPORTED, "more than 8192 features per frame");
    HIP_TRY(hipSetDevice(v->device));
    const size_t b_desc = up256((size_t)n * 32), b_i = up256((size_t)n * 4), b_o = up256((size_t)(n + 1) * 4),
                 b_d = up256((size_t)n * 8);
    const size_t stage = b_desc + b_i /*bow_word*/ + b_d /*bow_value*/ + b_i /*fv_node*/ + b_o /*fv_off*/ +
                         b_i /*fv_idx*/ + 256 /*counts*/;
    const size_t scratch = 2 * b_i + b_d;
    int rc = reserve_work(v, stage + scratch + 256);
    if (rc) return rc;
    char* w = v->work;
    uint8_t* d_desc = (uint8_t*)w;
    w += b_desc;
    int32_t* d_bw = (int32_t*)w;
    w += b_i;
    double* d_bv = (double*)w;
    w += b_d;
    int32_t* d_fn = (int32_t*)w;
    w += b_i;
    int32_t* d_fo = (int32_t*)w;
    w += b_o;
    int32_t* d_fi = (int32_t*)w;
    w += b_i;
    int32_t* d_cnt = (int32_t*)w;  // [0] = n, [1] = nbow, [2] = nfv
    w += 256;
    int32_t* d_word = (int32_t*)w;
    w += b_i;
    int32_t* d_node = (int32_t*)w;
    w += b_i;
    double* d_weight = (double*)w;
    HIP_TRY(hipMemcpyAsync(d_desc, desc, (size_t)n * 32, hipMemcpyHostToDevice, v->stream));
    HIP_TRY(hipMemcpyAsync(d_cnt, &n, 4, hipMemcpyHostToDevice, v->stream));
    rc = launch(v, 1, d_desc, d_cnt, n, levelsup, d_word, d_weight, d_node,
                FrameOut{d_bw, d_bv, d_cnt + 1, d_fn, d_fo, d_fi, d_cnt + 2}, v->stream, true);
    if (rc) return rc;
    int32_t cnt[3];
    HIP_TRY(hipMemcpyAsync(cnt, d_cnt, 12, hipMemcpyDeviceToHost, v->stream));
    HIP_TRY(hipStreamSynchronize(v->stream));
    const int nb = cnt[1], nf = cnt[2];
    HIP_TRY(hipMemcpyAsync(bow_word, d_bw, (size_t)nb * 4, hipMemcpyDeviceToHost, v->stream));
    HIP_TRY(hipMemcpyAsync(bow_value, d_bv, (size_t)nb * 8, hipMemcpyDeviceToHost, v->stream));
    HIP_TRY(hipMemcpyAsync(fv_node, d_fn, (size_t)nf * 4, hipMemcpyDeviceToHost, v->stream));
    HIP_TRY(hipMemcpyAsync(fv_off, d_fo, (size_t)(nf + 1) * 4, hipMemcpyDeviceToHost, v->stream));
    HIP_TRY(hipStreamSynchronize(v->stream));
    const int nw = fv_off[nf];
    HIP_TRY(hipMemcpy(fv_idx, d_fi, (size_t)nw * 4, hipMemcpyDeviceToHost));
    *nbow = nb;
    *nfv = nf;
    return ORBX_OK;
}

int orbx_vocabulary_set_timing(orbx_vocabulary* v, int enable) {
    if (!v) return fail(ORBX_ERR_ARG, "null vocabulary");
    v->timing = enable != 0;
    v->ncalls = 0;
    return ORBX_OK;
}

// Average over the (up to 64) most recent timed calls: [0] walk, [1] frame.
int orbx_vocabulary_stage_times(orbx_vocabulary* v, float* walk_ms, float* frame_ms) {
    if (!v || !walk_ms || !frame_ms) return fail(ORBX_ERR_ARG, "null argument");
    if (v->ncalls == 0) return fail(ORBX_ERR_STATE, "no timed transform yet");
    const long long last = v->ncalls - 1;
    const int nslots = v->ncalls < orbx_vocabulary::kRing ? (int)v->ncalls : orbx_vocabulary::kRing;
    HIP_TRY(hipEventSynchronize(v->ev[last % orbx_vocabulary::kRing][2]));
    double a = 0.0, b = 0.0;
    for (int k = 0; k < nslots; k++) {
        hipEvent_t* e = v->ev[(last - k) % orbx_vocabulary::kRing];
        float t0 = 0.f, t1 = 0.f;
        HIP_TRY(hipEventElapsedTime(&t0, e[0], e[1]));
        HIP_TRY(hipEventElapsedTime(&t1, e[1], e[2]));
        a += t0;
        b += t1;
    }
    *walk_ms = (float)(a / nslots);
    *frame_ms = (float)(b / nslots);
    return ORBX_OK;
}

}  // extern "C"
