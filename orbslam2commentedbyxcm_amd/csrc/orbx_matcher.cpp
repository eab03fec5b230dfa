// orbx_matcher.cpp -- host side of the ORBmatcher drop-in (include/orbx.h).
//
// Each entry point restates the reference function's object-graph walk on the host
// (projection of MapPoints, query filtering, vocabulary-node merge, row bands) and
// hands the dense part -- candidate windows, Hamming scoring, the ordered commit --
// to one kernel launch on the matcher's stream.  MapPoint* pointers are represented
// by integer ids; mvpMapPoints arrays hold ids (-1 = NULL).
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "orbx.h"
#include "orbx_error.h"
#include "orbx_kernels.h"

using namespace orbx;

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

constexpr int kNumCellsHost = kGridCols * kGridRows;
constexpr int TH_HIGH = 100;  // ORBmatcher.cc:38
constexpr int TH_LOW = 50;    // ORBmatcher.cc:39
constexpr long long kMaxMapPointIds = 1ll << 30;  // the searches carry a flag in bit 30 of a claim

// Grow-only device arena, reset per call.
struct Arena {
    char* base = nullptr;
    char* host = nullptr;  // pinned mirror: a call's inputs are staged here and uploaded in one copy
    char* host_dev = nullptr;  // the mirror's device address (mapped): a kernel can copy it in itself
    size_t cap = 0, used = 0, dirty = 0;
    hipError_t reserve(size_t bytes) {
        dirty = 0;
        if (bytes <= cap) return hipSuccess;
        if (base) (void)hipFree(base);
        if (host) (void)hipHostFree(host);
        base = host = host_dev = nullptr;
        cap = 0;
        bytes = (bytes + 15) & ~(size_t)15;
        hipError_t e = hipMalloc((void**)&base, bytes);
        if (e == hipSuccess) e = hipHostMalloc((void**)&host, bytes, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&host_dev, host, 0);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
    // the staged prefix for an in-kernel copy (instead of flush()): bytes, rounded to 16
    size_t take_staged() {
        const size_t b = (dirty + 15) & ~(size_t)15;
        dirty = 0;
        return b;
    }
    template <typename T>
    T* take(size_t n) {
        used = (used + 255) & ~(size_t)255;
        T* p = (T*)(base + used);
        used += sizeof(T) * (n ? n : 1);
        return p;
    }
    // stage `bytes` of host data for device address d (inside the arena)
    void up(void* d, const void* h, size_t bytes) {
        const size_t o = (size_t)((char*)d - base);
        std::memcpy(host + o, h, bytes);
        if (o + bytes > dirty) dirty = o + bytes;
    }
    // fill `bytes` at device address d with byte v, staged like up() (a device memset
    // before flush() would be overwritten by the prefix copy)
    void fill(void* d, int v, size_t bytes) {
        const size_t o = (size_t)((char*)d - base);
        std::memset(host + o, v, bytes);
        if (o + bytes > dirty) dirty = o + bytes;
    }
    // one upload of everything staged since the last flush (the prefix [0, dirty)): a copy
    // kernel reading the mapped mirror (a DMA copy's setup latency is most of a small
    // copy's cost; the GPU's own loads over PCIe are not)
    hipError_t flush(hipStream_t s) {
        if (!dirty) return hipSuccess;
        const hipError_t e = launch_stage_copy(host_dev, base, (dirty + 15) & ~(size_t)15, s);
        dirty = 0;
        return e;
    }
    // `bytes` at device address d (inside the arena) into the pinned mirror by a copy
    // kernel writing the mapped mirror; sync() copies it to h
    struct Pending { void* h; size_t o, bytes; };
    std::vector<Pending> pending;
    hipError_t down(void* h, const void* d, size_t bytes, hipStream_t s) {
        const size_t o = (size_t)((const char*)d - base);
        pending.push_back({h, o, bytes});
        return launch_stage_copy(d, host_dev + o, (bytes + 15) & ~(size_t)15, s);
    }
    hipError_t sync(hipStream_t s) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e == hipSuccess)
            for (const Pending& p : pending) std::memcpy(p.h, host + p.o, p.bytes);
        pending.clear();
        return e;
    }
    void release() {
        if (base) (void)hipFree(base);
        if (host) (void)hipHostFree(host);
        base = host = host_dev = nullptr;
        cap = used = dirty = 0;
    }
};

size_t pad(size_t b) { return ((b + 255) & ~(size_t)255) + 256; }

// Pinned staging for the asynchronous device calls' small host tables: a ring of slots,
// each reused only once the copy that last read it has run (its event), so a call never
// waits on the stream (a pageable hipMemcpyAsync would).
struct StageRing {
    static constexpr int kSlots = 4;
    char* host[kSlots] = {};
    size_t cap[kSlots] = {};
    hipEvent_t ev[kSlots] = {};
    bool pending[kSlots] = {};
    int next = 0;
    hipError_t get(size_t bytes, char** out, int* slot) {
        const int k = next;
        next = (next + 1) % kSlots;
        if (pending[k]) {
            const hipError_t e = hipEventSynchronize(ev[k]);
            if (e != hipSuccess) return e;
            pending[k] = false;
        }
        if (cap[k] < bytes) {
            if (host[k]) (void)hipHostFree(host[k]);
            host[k] = nullptr;
            cap[k] = 0;
            const hipError_t e = hipHostMalloc((void**)&host[k], bytes, hipHostMallocDefault);
            if (e != hipSuccess) return e;
            cap[k] = bytes;
        }
        if (!ev[k]) {
            const hipError_t e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
        *out = host[k];
        *slot = k;
        return hipSuccess;
    }
    hipError_t copied(int slot, hipStream_t s) {
        pending[slot] = true;
        return hipEventRecord(ev[slot], s);
    }
    void release() {
        for (int k = 0; k < kSlots; k++) {
            if (host[k]) (void)hipHostFree(host[k]);
            if (ev[k]) (void)hipEventDestroy(ev[k]);
            host[k] = nullptr;
            ev[k] = nullptr;
            cap[k] = 0;
            pending[k] = false;
        }
    }
};

// x_c = R x + t, float products summed left to right (gemm accumulation unpinned)
void project(const float* Tcw, const float* X, float* xc) {
    for (int r = 0; r < 3; r++)
        xc[r] = Tcw[4 * r] * X[0] + Tcw[4 * r + 1] * X[1] + Tcw[4 * r + 2] * X[2] + Tcw[4 * r + 3];
}

// camera centre -R^T t
void centre(const float* Tcw, float* c) {
    for (int k = 0; k < 3; k++) c[k] = -(Tcw[k] * Tcw[3] + Tcw[4 + k] * Tcw[7] + Tcw[8 + k] * Tcw[11]);
}

// cv::norm of a 3x1 CV_32F Mat: squares accumulated in double, sqrt, stored as float
float norm3(const float* p) {
    double s = 0.0;
    for (int k = 0; k < 3; k++) s += (double)p[k] * p[k];
    return (float)std::sqrt(s);
}

// MapPoint::PredictScale (MapPoint.cc:469-509): C log(double) of the float ratio (no
// `using namespace std` there), double quotient, ceil; mfLogScaleFactor = (float)log(sf).
int predict_scale(float max_distance, float current_dist, const orbx_frame_view* f) {
    const float ratio = max_distance / current_dist;
    const float log_scale = (float)std::log((double)f->scale_factors[1]);
    int n = (int)std::ceil(std::log((double)ratio) / (double)log_scale);
    if (n < 0) n = 0;
    else if (n >= f->nlevels) n = f->nlevels - 1;
    return n;
}

}  // namespace

struct orbx_matcher {
    int device = 0;
    float nnratio = 0.6f;
    int check_ori = 1;
    hipStream_t stream = nullptr;
    Arena arena;
    // orbx_match_sequence_device timing: a ring of (start, end) events, one per timed
    // call, averaged by orbx_matcher_last_ms.
    static constexpr int kRing = 64;
    bool timing = false;
    hipEvent_t ev[kRing][2] = {};
    long long ncalls = 0;
    int footprint = 0;  // orbx_matcher_set_footprint: 0 full, 1 small, 2 split, 3 one wave, 4 lean, 5 lean split
    // device-only scratch of the batched device calls (no pinned mirror)
    char* dscr = nullptr;
    size_t dscr_cap = 0;
    // tables of orbx_search_for_triangulation_batch_device (device-only)
    char* tscr = nullptr;
    size_t tscr_cap = 0;
    // queries, problems and grids of orbx_search_local_points_device (device-only)
    char* lscr = nullptr;
    size_t lscr_cap = 0;
    StageRing stage;
    // wall time of the newest drop-in host call (entry to return), as a C++ caller sees it
    double last_call_us = 0.0;
    // host-mapped pinned results of the single projection calls (mvpMapPoints + count):
    // the commit kernel writes them over PCIe, so a call needs no device-to-host copy
    int32_t* hmp = nullptr;
    int32_t* hmp_dev = nullptr;
    size_t hmp_cap = 0;
};

namespace {
// Scoped: stores the enclosing host call's wall time in m->last_call_us.
struct CallClock {
    orbx_matcher* m;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit CallClock(orbx_matcher* mm) : m(mm) {}
    ~CallClock() {
        if (m) m->last_call_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
};
}  // namespace

namespace {

// Upload one frame view + queries and run k_proj_search for a single problem.
int run_proj(orbx_matcher* m, const orbx_frame_view* f, int32_t* frame_mp, const std::vector<ProjQuery>& qs,
             const std::vector<uint8_t>& qdesc, const orbx_mappoints* mps, const ProjParams& base_params,
             int* nmatches, int replay_rt = 0) {
    const int n = f->n, nq = (int)qs.size();
    if (nq == 0 || n == 0) {
        if (nmatches) *nmatches = 0;
        return ORBX_OK;
    }
    if (mps->n < 0 || mps->n >= kMaxMapPointIds) return fail(ORBX_ERR_ARG, "MapPoint table of 2^30 or more");
    const auto t_stage0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(m->device));
    const int nobs = mps->n;
    size_t need = pad(sizeof(orbx_keypoint) * n) + pad((size_t)n * 32) + pad(sizeof(float) * n) +
                  pad(sizeof(int32_t) * n) + pad(sizeof(ProjQuery) * nq) + pad((size_t)nq * 32) +
                  pad(sizeof(int32_t) * (nobs ? nobs : 1)) + pad(sizeof(ProjProblem)) + pad(8 * kProjScratchWords * (size_t)nq) +
                  pad(sizeof(long long)) + pad(sizeof(int32_t));
    // one problem: the split launches (grid sort, scoring spread over nq / 16 workgroups,
    // one-wave commit) finish sooner than one workgroup doing all three
    const int gcap = n > nq ? n : nq;
    // octave buckets of the device grid: one per octave present (the grid keys hold
    // octave & 31)
    int noct = 1;
    for (int i = 0; i < n; i++) {
        const int o = f->keys[i].octave & 31;
        if (o + 1 > noct) noct = o + 1;
    }
    need += pad(seq_grid_bytes(gcap, noct));
    HIP_TRY(m->arena.reserve(need));
    m->arena.used = 0;
    auto* d_keys = m->arena.take<orbx_keypoint>(n);
    auto* d_desc = m->arena.take<uint8_t>((size_t)n * 32);
    auto* d_ur = m->arena.take<float>(n);
    auto* d_fmp = m->arena.take<int32_t>(n);
    auto* d_q = m->arena.take<ProjQuery>(nq);
    auto* d_qd = m->arena.take<uint8_t>((size_t)nq * 32);
    auto* d_obs = m->arena.take<int32_t>(nobs ? nobs : 1);
    auto* d_prob = m->arena.take<ProjProblem>(1);
    auto* d_off = m->arena.take<long long>(1);
    auto* d_nm = m->arena.take<int32_t>(1);
    // device-only areas last: the staged (uploaded) prefix ends before them
    auto* d_scr = m->arena.take<unsigned long long>(kProjScratchWords * (size_t)nq);
    auto* d_grid = m->arena.take<unsigned char>(seq_grid_bytes(gcap, noct));
    hipStream_t s = m->stream;
    m->arena.up(d_keys, f->keys, sizeof(orbx_keypoint) * n);
    m->arena.up(d_desc, f->desc, (size_t)n * 32);
    if (f->u_right) m->arena.up(d_ur, f->u_right, sizeof(float) * n);
    m->arena.up(d_fmp, frame_mp, sizeof(int32_t) * n);
    m->arena.up(d_q, qs.data(), sizeof(ProjQuery) * nq);
    m->arena.up(d_qd, qdesc.data(), (size_t)nq * 32);
    if (nobs && mps->observations)
        m->arena.up(d_obs, mps->observations, sizeof(int32_t) * nobs);
    ProjProblem pb{};
    pb.keys = d_keys;
    pb.desc = d_desc;
    pb.u_right = f->u_right ? d_ur : nullptr;
    pb.frame_mp = d_fmp;
    pb.n = n;
    pb.q = d_q;
    pb.qdesc = d_qd;
    pb.nq = nq;
    pb.min_x = f->min_x;
    pb.min_y = f->min_y;
    pb.inv_w = (float)kGridCols / (f->max_x - f->min_x);  // Frame.cc:157-159
    pb.inv_h = (float)kGridRows / (f->max_y - f->min_y);
    pb.nmatches = d_nm;
    const long long zero = 0;
    m->arena.up(d_prob, &pb, sizeof(pb));
    m->arena.up(d_off, &zero, sizeof(zero));
    ProjParams P = base_params;
    P.mp_obs = d_obs;
    P.noct = noct;
    // switch call_stamps = 1: the call's host phases and the replay's counters to stderr
    // (diagnostics only)
    const bool call_stamps = tuning(Tune::CallStamps, 0) > 0;
    unsigned long long* d_st = nullptr;
    const auto t_flush = std::chrono::steady_clock::now();
    if (call_stamps) {
        HIP_TRY(hipMalloc(&d_st, sizeof(unsigned long long) * kStampWords));
        HIP_TRY(hipMemsetAsync(d_st, 0, sizeof(unsigned long long) * kStampWords, s));
        P.stamps = d_st;
    }
    // results straight into host-mapped memory (k_seq_commit's out_mp and the count)
    const bool mapped = gcap < 8192;
    if (mapped && m->hmp_cap < (size_t)n + 1) {
        HIP_TRY(hipStreamSynchronize(s));
        if (m->hmp) (void)hipHostFree(m->hmp);
        m->hmp = m->hmp_dev = nullptr;
        m->hmp_cap = 0;
        // coherent explicitly: the kernel's stores must be visible to the memcpy after the
        // stream synchronise whatever the runtime's default coherence setting
        HIP_TRY(hipHostMalloc((void**)&m->hmp, sizeof(int32_t) * ((size_t)n + 1),
                              hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer((void**)&m->hmp_dev, m->hmp, 0));
        m->hmp_cap = (size_t)n + 1;
    }
    if (mapped) {
        P.out_mp = m->hmp_dev + 1;
        pb.nmatches = m->hmp_dev;
        m->arena.up(d_prob, &pb, sizeof(pb));
    }
    if (mapped) {
        // inputs copied in by k_stage_copy (no DMA), results written to mapped memory
        const size_t staged = m->arena.take_staged();
        // replay width: the row's (replay_rt) unless switch replay_threads overrides it
        const bool rt_env = tuning(Tune::ReplayThreads, 0) > 0;
        HIP_TRY(launch_seq_split(d_prob, 1, P, d_grid, gcap, d_scr, d_off, s, 0, rt_env ? 0 : replay_rt,
                                 m->arena.host_dev, m->arena.base, staged));
    } else {
        HIP_TRY(m->arena.flush(s));
        HIP_TRY(launch_proj_search(d_prob, 1, P, d_scr, d_off, n, nq, s));
    }
    // the caller's frame_mp is written only once the count says the replay converged: a
    // failed call (ORBX_ERR_STATE below) leaves it as it was
    int nm = 0;
    std::vector<int32_t> staged_mp;
    if (!mapped) {
        staged_mp.resize((size_t)n);
        HIP_TRY(m->arena.down(staged_mp.data(), d_fmp, sizeof(int32_t) * n, s));
        HIP_TRY(m->arena.down(&nm, d_nm, sizeof(int32_t), s));
    }
    const auto t_enq = std::chrono::steady_clock::now();
    HIP_TRY(m->arena.sync(s));
    if (mapped) nm = m->hmp[0];
    if (nm >= 0) std::memcpy(frame_mp, mapped ? m->hmp + 1 : staged_mp.data(), sizeof(int32_t) * n);
    if (call_stamps) {
        const auto t_done = std::chrono::steady_clock::now();
        unsigned long long h[kStampWords];
        HIP_TRY(hipMemcpy(h, d_st, sizeof(h), hipMemcpyDeviceToHost));
        HIP_TRY(hipFree(d_st));
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        fprintf(stderr, "[orbx call] n=%d nq=%d | host staging %.1f us, enqueue %.1f us, wait %.1f us | grid: start %.1f, "
                "sort %.1f, writes %.1f, colstart %.1f, runs %.1f us | replay (%llu threads) %.1f us, %llu iterations, "
                "%llu re-scored (%.1f us), ",
                n, nq, us(t_stage0, t_flush), us(t_flush, t_enq), us(t_enq, t_done), (double)(h[1] - h[0]) * 0.01,
                (double)(h[2] - h[1]) * 0.01, (double)(h[4] - h[2]) * 0.01, (double)(h[10] - h[4]) * 0.01,
                (double)(h[11] - h[10]) * 0.01, h[kStampForm], (double)(h[3] - h[13]) * 0.01, h[7], h[5],
                (double)h[8] * 0.01);
        if (h[kStampForm] == 64)  // one wave: 9 = loads + first rounds (cumulative), 15 = a clock reading
            fprintf(stderr, "chunk loads %.1f + first rounds %.1f us, after the loop %.1f us\n", (double)h[14] * 0.01,
                    h[9] >= h[14] ? (double)(h[9] - h[14]) * 0.01 : 0.0,
                    h[15] && h[3] >= h[15] ? (double)(h[3] - h[15]) * 0.01 : 0.0);
        else  // block replay: 9 / 14 / 15 are durations
            fprintf(stderr, "chunk loads %.1f, rounds %.1f, commits %.1f us\n", (double)h[14] * 0.01,
                    (double)h[9] * 0.01, (double)h[15] * 0.01);
    }
    if (nm < 0)  // the replay's iteration guard fired: frame_mp is partial, never report it as matches
        return fail(ORBX_ERR_STATE, "SearchByProjection replay did not converge (iteration guard)");
    if (nmatches) *nmatches = nm;
    return ORBX_OK;
}

}  // namespace

extern "C" {

int orbx_matcher_create(int device, float nnratio, int check_ori, orbx_matcher** out) {
    if (!out) return fail(ORBX_ERR_ARG, "null out");
    *out = nullptr;
    orbx_matcher* m = new (std::nothrow) orbx_matcher();
    if (!m) return fail(ORBX_ERR_ARG, "out of host memory");
    m->device = device;
    m->nnratio = nnratio;
    m->check_ori = check_ori ? 1 : 0;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete m;
        set_last_error(std::string("orbx_matcher_create: ") + hipGetErrorString(e));
        return ORBX_ERR_HIP;
    }
    *out = m;
    return ORBX_OK;
}

void orbx_matcher_destroy(orbx_matcher* m) {
    if (!m || orbx::unloading()) return;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    m->arena.release();
    if (m->dscr) (void)hipFree(m->dscr);
    if (m->tscr) (void)hipFree(m->tscr);
    if (m->lscr) (void)hipFree(m->lscr);
    m->stage.release();
    if (m->hmp) (void)hipHostFree(m->hmp);
    for (auto& slot : m->ev)
        for (auto& e : slot)
            if (e) (void)hipEventDestroy(e);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

// ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th), ORBmatcher.cc:61-173
int orbx_search_by_projection_local(orbx_matcher* m, const orbx_frame_view* f, int32_t* frame_mp,
                                    const int32_t* queries, int nq, const orbx_mappoints* mps, const orbx_track* trk,
                                    float th, int* nmatches) {
    const CallClock clock_(m);
    if (!m || !f || !frame_mp || !mps || !trk || (nq && !queries)) return fail(ORBX_ERR_ARG, "null argument");
    const bool bFactor = th != 1.0;  // ORBmatcher.cc:66
    std::vector<ProjQuery> qs;
    std::vector<uint8_t> qd;
    qs.reserve(nq);
    qd.reserve((size_t)nq * 32);
    for (int i = 0; i < nq; i++) {
        const int mp = queries[i];
        if (mp < 0 || mp >= mps->n) return fail(ORBX_ERR_ARG, "MapPoint id out of range");
        if (!trk->in_view[mp]) continue;
        if (mps->bad && mps->bad[mp]) continue;
        const int pred = trk->scale_level[mp];
        if (pred < 0 || pred >= f->nlevels) return fail(ORBX_ERR_ARG, "predicted level out of range");
        float r = trk->view_cos[mp] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos, ORBmatcher.cc:176-183
        if (bFactor) r *= th;
        ProjQuery q{};
        q.u = trk->proj_x[mp];
        q.v = trk->proj_y[mp];
        q.ur = trk->proj_xr[mp];
        q.r = r * f->scale_factors[pred];
        q.er_max = r * f->scale_factors[pred];
        q.min_level = pred - 1;
        q.max_level = pred;
        q.post_min = -1;
        q.post_max = -1;
        q.mp = mp;
        q.angle = 0.f;
        qs.push_back(q);
        qd.insert(qd.end(), mps->desc + (size_t)mp * 32, mps->desc + (size_t)mp * 32 + 32);
    }
    ProjParams P{};
    P.blocked_mode = 0;
    P.accept_th = TH_HIGH;
    P.ratio_mode = 1;
    P.nnratio = m->nnratio;
    P.check_ori = 0;
    return run_proj(m, f, frame_mp, qs, qd, mps, P, nmatches);
}

// ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono), ORBmatcher.cc:1620-1789
int orbx_search_by_projection_frame(orbx_matcher* m, const orbx_frame_view* cur, int32_t* cur_mp,
                                    const orbx_frame_view* last, const int32_t* last_mp, const uint8_t* last_outlier,
                                    const orbx_mappoints* mps, float th, int mono, int* nmatches) {
    const CallClock clock_(m);
    if (!m || !cur || !cur_mp || !last || !last_mp || !mps || !mps->pos) return fail(ORBX_ERR_ARG, "null argument");
    float twc[3], tlc[3];
    centre(cur->Tcw, twc);       // twc = -Rcw^T tcw (cc:1637)
    project(last->Tcw, twc, tlc);  // tlc = Rlw*twc + tlw (cc:1643)
    const bool bForward = tlc[2] > cur->b && !mono;
    const bool bBackward = -tlc[2] > cur->b && !mono;
    std::vector<ProjQuery> qs;
    std::vector<uint8_t> qd;
    for (int i = 0; i < last->n; i++) {
        const int mp = last_mp[i];
        if (mp < 0) continue;
        if (mp >= mps->n) return fail(ORBX_ERR_ARG, "MapPoint id out of range");
        if (last_outlier && last_outlier[i]) continue;
        float x3Dc[3];
        project(cur->Tcw, mps->pos + 3 * (size_t)mp, x3Dc);
        const float xc = x3Dc[0], yc = x3Dc[1];
        const float invzc = (float)(1.0 / x3Dc[2]);
        if (invzc < 0) continue;
        // fused as g++ -O3 -march=native builds the reference (H4)
        const float u = std::fma(cur->fx * xc, invzc, cur->cx);
        const float v = std::fma(cur->fy * yc, invzc, cur->cy);
        if (u < cur->min_x || u > cur->max_x) continue;
        if (v < cur->min_y || v > cur->max_y) continue;
        const int nLastOctave = last->keys[i].octave;
        const float radius = th * cur->scale_factors[nLastOctave];
        ProjQuery q{};
        q.u = u;
        q.v = v;
        q.ur = std::fma(-cur->bf, invzc, u);
        q.r = radius;
        q.er_max = radius;
        if (bForward) {
            q.min_level = nLastOctave;
            q.max_level = -1;
        } else if (bBackward) {
            q.min_level = 0;
            q.max_level = nLastOctave;
        } else {
            q.min_level = nLastOctave - 1;
            q.max_level = nLastOctave + 1;
        }
        q.post_min = -1;
        q.post_max = -1;
        q.mp = mp;
        q.angle = last->keys[i].angle;
        qs.push_back(q);
        qd.insert(qd.end(), mps->desc + (size_t)mp * 32, mps->desc + (size_t)mp * 32 + 32);
    }
    ProjParams P{};
    P.blocked_mode = 0;
    P.accept_th = TH_HIGH;
    P.ratio_mode = 0;
    P.check_ori = m->check_ori;
    return run_proj(m, cur, cur_mp, qs, qd, mps, P, nmatches);
}

// ORBmatcher::SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist),
// ORBmatcher.cc:1792-1924: queries in KeyFrame keypoint order; any assigned keypoint of
// the current frame is skipped (cc:1865-1866); best <= ORBdist; rotation check.
int orbx_search_by_projection_keyframe(orbx_matcher* m, const orbx_frame_view* cur, int32_t* cur_mp,
                                       const orbx_frame_view* kf, const int32_t* kf_mp,
                                       const uint8_t* already_found, const orbx_mappoints* mps, float th,
                                       int orb_dist, int* nmatches) {
    const CallClock clock_(m);
    if (!m || !cur || !cur_mp || !kf || !kf_mp || !mps || !mps->pos || !mps->max_distance || !mps->min_distance)
        return fail(ORBX_ERR_ARG, "null argument");
    if (cur->nlevels < 2) return fail(ORBX_ERR_ARG, "need >= 2 pyramid levels");
    float Ow[3];
    centre(cur->Tcw, Ow);  // cc:1796-1798
    std::vector<ProjQuery> qs;
    std::vector<uint8_t> qd;
    for (int i = 0; i < kf->n; i++) {
        const int mp = kf_mp[i];
        if (mp < 0) continue;
        if (mp >= mps->n) return fail(ORBX_ERR_ARG, "MapPoint id out of range");
        if (mps->bad && mps->bad[mp]) continue;
        if (already_found && already_found[mp]) continue;
        const float* x3Dw = mps->pos + 3 * (size_t)mp;
        float x3Dc[3];
        project(cur->Tcw, x3Dw, x3Dc);
        const float invzc = (float)(1.0 / x3Dc[2]);
        const float u = std::fma(cur->fx * x3Dc[0], invzc, cur->cx);  // fused (H4)
        const float v = std::fma(cur->fy * x3Dc[1], invzc, cur->cy);
        if (u < cur->min_x || u > cur->max_x) continue;
        if (v < cur->min_y || v > cur->max_y) continue;
        float PO[3];
        for (int c = 0; c < 3; c++) PO[c] = x3Dw[c] - Ow[c];
        const float dist3D = norm3(PO);
        if (dist3D < 0.8f * mps->min_distance[mp] || dist3D > 1.2f * mps->max_distance[mp]) continue;
        const int pred = predict_scale(mps->max_distance[mp], dist3D, cur);
        ProjQuery q{};
        q.u = u;
        q.v = v;
        q.r = th * cur->scale_factors[pred];
        q.er_max = -1.f;
        q.min_level = pred - 1;  // GetFeaturesInArea(u, v, radius, pred-1, pred+1)
        q.max_level = pred + 1;
        q.post_min = -1;
        q.post_max = -1;
        q.mp = mp;
        q.angle = kf->keys[i].angle;
        qs.push_back(q);
        qd.insert(qd.end(), mps->desc + (size_t)mp * 32, mps->desc + (size_t)mp * 32 + 32);
    }
    ProjParams P{};
    P.blocked_mode = 1;
    P.accept_th = orb_dist;
    P.ratio_mode = 0;
    P.check_ori = m->check_ori;
    // a 1024-thread replay: this row's conflict chains are short (r03 rows: 29 one-wave
    // iterations against a12's 109), so a wider fixpoint finishes sooner
    return run_proj(m, cur, cur_mp, qs, qd, mps, P, nmatches, 1024);
}

// ORBmatcher::SearchByProjection(KeyFrame*, cv::Mat Scw, const vector<MapPoint*>&,
// vector<MapPoint*>&, int th), ORBmatcher.cc:398-520.  OpenCV arithmetic as restated in
// DESIGN.md §2 (Mat::dot in double, Mat / s as a float multiply by (float)(1/s)).
int orbx_search_by_projection_sim3(orbx_matcher* m, const orbx_frame_view* kf, const float* Scw,
                                   const int32_t* points, int npoints, int32_t* matched,
                                   const orbx_mappoints* mps, int th, int* nmatches) {
    const CallClock clock_(m);
    if (!m || !kf || !Scw || !matched || !mps || !mps->pos || !mps->max_distance || !mps->min_distance ||
        !mps->normal || (npoints && !points))
        return fail(ORBX_ERR_ARG, "null argument");
    if (kf->nlevels < 2) return fail(ORBX_ERR_ARG, "need >= 2 pyramid levels");
    double d0 = 0.0;
    for (int c = 0; c < 3; c++) d0 += (double)Scw[c] * Scw[c];
    const float scw = (float)std::sqrt(d0);                 // cc:408
    const float alpha = (float)(1.0 / scw);
    float T[12];                                            // Rcw = sRcw / scw, tcw = st / scw (cc:409-410)
    for (int k = 0; k < 12; k++) T[k] = Scw[k] * alpha;
    float Ow[3];
    centre(T, Ow);                                          // cc:411
    std::vector<uint8_t> found((size_t)(mps->n > 0 ? mps->n : 1), 0);  // spAlreadyFound (cc:414-415)
    for (int i = 0; i < kf->n; i++) {
        if (matched[i] >= mps->n) return fail(ORBX_ERR_ARG, "MapPoint id out of range");
        if (matched[i] >= 0) found[matched[i]] = 1;
    }
    std::vector<ProjQuery> qs;
    std::vector<uint8_t> qd;
    for (int k = 0; k < npoints; k++) {
        const int mp = points[k];
        if (mp < 0 || mp >= mps->n) return fail(ORBX_ERR_ARG, "MapPoint id out of range");
        if ((mps->bad && mps->bad[mp]) || found[mp]) continue;
        const float* p3Dw = mps->pos + 3 * (size_t)mp;
        float p3Dc[3];
        project(T, p3Dw, p3Dc);
        if (p3Dc[2] < 0.0) continue;
        const float invz = 1 / p3Dc[2];
        const float u = std::fma(kf->fx, p3Dc[0] * invz, kf->cx);  // fused (H4)
        const float v = std::fma(kf->fy, p3Dc[1] * invz, kf->cy);
        if (!(u >= kf->min_x && u < kf->max_x && v >= kf->min_y && v < kf->max_y)) continue;  // IsInImage
        float PO[3];
        for (int c = 0; c < 3; c++) PO[c] = p3Dw[c] - Ow[c];
        const float dist = norm3(PO);
        if (dist < 0.8f * mps->min_distance[mp] || dist > 1.2f * mps->max_distance[mp]) continue;
        const float* Pn = mps->normal + 3 * (size_t)mp;
        double dot = 0.0;
        for (int c = 0; c < 3; c++) dot += (double)PO[c] * Pn[c];
        if (dot < 0.5 * dist) continue;
        const int pred = predict_scale(mps->max_distance[mp], dist, kf);
        ProjQuery q{};
        q.u = u;
        q.v = v;
        q.r = (float)th * kf->scale_factors[pred];
        q.er_max = -1.f;
        q.min_level = -1;  // KeyFrame::GetFeaturesInArea has no level arguments
        q.max_level = -1;
        q.post_min = pred - 1;  // kpLevel in [pred-1, pred] (cc:480-483)
        q.post_max = pred;
        q.mp = mp;
        q.angle = 0.f;
        qs.push_back(q);
        qd.insert(qd.end(), mps->desc + (size_t)mp * 32, mps->desc + (size_t)mp * 32 + 32);
    }
    ProjParams P{};
    P.blocked_mode = 1;
    P.accept_th = TH_LOW;
    P.ratio_mode = 0;
    P.check_ori = 0;
    // short conflict chains (accept <= TH_LOW; 17 one-wave iterations): 1024-thread replay
    return run_proj(m, kf, matched, qs, qd, mps, P, nmatches, 1024);
}

// Batched SearchByProjection(CurrentFrame, LastFrame, th, bMono) over a device
// sequence written by orbx_extract_batch_device (see include/orbx.h).
int orbx_match_sequence_device(orbx_matcher* m, int batch, const orbx_keypoint* d_kps, const uint8_t* d_desc,
                               const int32_t* d_n, int cap, const float* d_Tcw, float fx, float fy, float cx,
                               float cy, float min_x, float max_x, float min_y, float max_y,
                               const float* scale_factors, int nlevels, float depth, float th, int32_t* d_cur_mp,
                               int32_t* d_nmatches, void* stream) {
    orbx_sequence q{};
    q.batch = batch;
    q.kps = d_kps;
    q.desc = d_desc;
    q.n = d_n;
    q.cap = cap;
    q.Tcw = d_Tcw;
    q.depth = depth;
    q.fx = fx;
    q.fy = fy;
    q.cx = cx;
    q.cy = cy;
    q.min_x = min_x;
    q.max_x = max_x;
    q.min_y = min_y;
    q.max_y = max_y;
    q.nlevels = nlevels;
    q.scale_factors = scale_factors;
    q.th = th;
    q.mono = 1;
    q.cur_mp = d_cur_mp;
    q.nmatches = d_nmatches;
    return orbx_match_sequence_device_ex(m, &q, stream);
}

int orbx_match_sequence_device_ex(orbx_matcher* m, const orbx_sequence* sq, void* stream) {
    if (!m || !sq) return fail(ORBX_ERR_ARG, "null argument");
    const int batch = sq->batch, cap = sq->cap, nlevels = sq->nlevels;
    if (batch < 0 || cap <= 0 || !sq->scale_factors || nlevels < 1 || nlevels > 32)
        return fail(ORBX_ERR_ARG, "bad argument");
    if (batch == 0) return ORBX_OK;
    if (!sq->kps || !sq->desc || !sq->n || !sq->Tcw || !sq->cur_mp || !sq->nmatches)
        return fail(ORBX_ERR_ARG, "null buffer");
    if ((long long)batch * cap >= kMaxMapPointIds) return fail(ORBX_ERR_ARG, "batch x cap MapPoint ids >= 2^30");
    if (!sq->mono && !(sq->b > 0.f)) return fail(ORBX_ERR_ARG, "stereo / RGB-D sequence needs the baseline mb > 0");
    if (sq->mp_obs && !sq->global_ids) return fail(ORBX_ERR_ARG, "mp_obs is indexed by global MapPoint ids");
    if (sq->retry_below < 0) return fail(ORBX_ERR_ARG, "retry_below must be >= 0");
    int32_t* d_cur_mp = sq->cur_mp;
    int32_t* d_nmatches = sq->nmatches;
    HIP_TRY(hipSetDevice(m->device));
    hipStream_t s = stream ? (hipStream_t)stream : m->stream;
    const int npairs = batch - 1;
    const bool split = m->footprint == 2;
    const bool grids = split || m->footprint == 5;  // a global grid area per problem
    const size_t np1 = (size_t)(npairs > 0 ? npairs : 1);
    const size_t need = pad(sizeof(ProjQuery) * np1 * cap) + pad(sizeof(ProjProblem) * np1) +
                        pad(sizeof(long long) * np1) + pad(sizeof(unsigned long long) * kProjScratchWords * np1 * cap) +
                        (grids ? pad(seq_grid_bytes(cap, nlevels) * np1) : 0);
    if (m->arena.cap < need) {
        HIP_TRY(hipStreamSynchronize(s));
        HIP_TRY(m->arena.reserve(need));
    }
    m->arena.used = 0;
    auto* d_q = m->arena.take<ProjQuery>((size_t)(npairs > 0 ? npairs : 1) * cap);
    auto* d_prob = m->arena.take<ProjProblem>(npairs > 0 ? npairs : 1);
    auto* d_off = m->arena.take<long long>(npairs > 0 ? npairs : 1);
    auto* d_scr = m->arena.take<unsigned long long>(kProjScratchWords * (size_t)(npairs > 0 ? npairs : 1) * cap);
    auto* d_grids = grids ? m->arena.take<unsigned char>(seq_grid_bytes(cap, nlevels) * np1) : nullptr;
    if (npairs == 0) {  // otherwise k_seq_build initialises both outputs
        HIP_TRY(hipMemsetAsync(d_cur_mp, 0xff, sizeof(int32_t) * (size_t)batch * cap, s));
        HIP_TRY(hipMemsetAsync(d_nmatches, 0, sizeof(int32_t) * (size_t)batch, s));
        return ORBX_OK;
    }
    SeqArgs A{};
    A.kps = sq->kps;
    A.desc = sq->desc;
    A.n = sq->n;
    A.cap = cap;
    A.Tcw = sq->Tcw;
    A.u_right = sq->u_right;
    A.mp_pos = sq->mp_pos;
    A.has_mp = sq->has_mp;
    A.fx = sq->fx;
    A.fy = sq->fy;
    A.cx = sq->cx;
    A.cy = sq->cy;
    A.bf = sq->bf;
    A.b = sq->b;
    A.min_x = sq->min_x;
    A.max_x = sq->max_x;
    A.min_y = sq->min_y;
    A.max_y = sq->max_y;
    A.depth = sq->depth;
    A.mono = sq->mono ? 1 : 0;
    A.global_ids = sq->global_ids ? 1 : 0;
    A.th = sq->th;
    for (int l = 0; l < nlevels; l++) A.scale[l] = sq->scale_factors[l];
    A.cur_mp = d_cur_mp;
    A.nmatches = d_nmatches;
    hipEvent_t* ev = m->ev[m->ncalls % orbx_matcher::kRing];
    if (m->timing) {
        for (int i = 0; i < 2; i++)
            if (!ev[i]) HIP_TRY(hipEventCreate(&ev[i]));
        HIP_TRY(hipEventRecord(ev[0], s));
    }
    HIP_TRY(launch_seq_build(A, npairs, d_q, d_prob, d_off, s));
    ProjParams P{};
    // without mp_obs every MapPoint of the sequence has Observations() > 0; with it a claim
    // blocks only when the claiming MapPoint's does (ORBmatcher.cc:1716-1718)
    P.mp_obs = sq->mp_obs;
    P.blocked_mode = sq->mp_obs ? 0 : 1;
    P.accept_th = TH_HIGH;
    P.ratio_mode = 0;
    P.check_ori = m->check_ori;
    P.noct = nlevels;  // the extractor's keypoints have octave < nlevels
    // ORBX_MATCH_STAMPS=1: per-phase wall-clock breakdown of the search kernel to stderr
    // (diagnostics only; synchronises the stream).
    // (with grids -- the split launches and the lean form -- the commit kernel's replay only)
    const bool stamps = tuning(Tune::MatchStamps, 0) > 0;
    unsigned long long* d_st = nullptr;
    if (stamps) {
        HIP_TRY(hipMalloc(&d_st, sizeof(unsigned long long) * kStampWords * npairs));
        HIP_TRY(hipMemsetAsync(d_st, 0, sizeof(unsigned long long) * kStampWords * npairs, s));
        P.stamps = d_st;
    }
    if (split) {
        HIP_TRY(launch_seq_split(d_prob, npairs, P, d_grids, cap, d_scr, d_off, s));
    } else {
        HIP_TRY(launch_proj_search(d_prob, npairs, P, d_scr, d_off, cap, cap, s, m->footprint == 1,
                                   m->footprint == 3, m->footprint == 4, m->footprint == 5 ? d_grids : nullptr));
    }
    if (sq->retry_below > 0) {
        // Tracking::TrackWithMotionModel (Tracking.cc:988-994): pairs left with fewer than
        // retry_below matches are searched again at 2*th.  The gate is read on the device
        // (k_seq_build), so nothing synchronises; the skipped pairs' workgroups leave at
        // once.  One launch of the one-wave form (sort, scoring and replay in one wave per
        // pair, the smallest footprint): the retried pairs are rare, and what the common case
        // pays is getting the launch's workgroups onto CUs the extraction keeps busy -- the
        // lean 1024-thread form took 282 us per launch there to skip every pair (r06d trace).
        A.retry_below = sq->retry_below;
        A.th = 2.f * sq->th;
        HIP_TRY(launch_seq_build(A, npairs, d_q, d_prob, d_off, s));
        HIP_TRY(launch_proj_search(d_prob, npairs, P, d_scr, d_off, cap, cap, s, false, true, false, nullptr));
    }
    if (m->timing) {
        HIP_TRY(hipEventRecord(ev[1], s));
        m->ncalls++;
    }
    if (stamps) {
        std::vector<unsigned long long> h((size_t)kStampWords * npairs);
        HIP_TRY(hipStreamSynchronize(s));
        HIP_TRY(hipMemcpy(h.data(), d_st, h.size() * 8, hipMemcpyDeviceToHost));
        HIP_TRY(hipFree(d_st));
        if (grids) {
            double cm = 0, cmx = 0, resc = 0, nq = 0, nit = 0, itmx = 0, sc = 0, gr = 0;
            double tl = 0, tr = 0, tcm = 0, trs = 0, nst = 0;
            for (int p = 0; p < npairs; p++) {
                const unsigned long long* r = &h[(size_t)kStampWords * p];
                if (!split) {  // the lean form's search kernel: grid, then scoring
                    gr += (double)(r[1] - r[0]) * 0.01;
                    sc += (double)(r[2] - r[1]) * 0.01;
                }
                const double d = (double)(r[3] - r[13]) * 0.01;
                tl += (double)r[14] * 0.01;
                if (r[kStampForm] == 64) {  // one-wave replay: 9 = loads + first rounds; no commit duration
                    tr += (double)(r[9] >= r[14] ? r[9] - r[14] : 0) * 0.01;
                } else {  // block replay: rounds and commits as durations
                    tr += (double)r[9] * 0.01;
                    tcm += (double)r[15] * 0.01;
                }
                trs += (double)r[8] * 0.01;
                nst += (double)r[12];
                cm += d;
                cmx = d > cmx ? d : cmx;
                resc += (double)r[5];
                nq += (double)r[6];
                nit += (double)r[7];
                itmx = (double)r[7] > itmx ? (double)r[7] : itmx;
            }
#if ORBX_SCORE_COUNT
            {
                double a = 0, b = 0, c = 0, n = 0, gm = 0, wm = 0;
                for (int p = 0; p < npairs; p++) {
                    const unsigned long long* r = &h[(size_t)kStampWords * p];
                    a += (double)r[kStampScore];
                    b += (double)r[kStampScore + 1];
                    c += (double)r[kStampScore + 2];
                    n += (double)r[kStampScore + 3];
                    gm += (double)r[kStampScore + 4];
                    wm += (double)r[kStampScore + 5];
                }
                fprintf(stderr, "[orbx score counts] per scored query: %.1f (column, octave) visits, %.1f entry steps, "
                        "%.1f candidates in the window (summed over the query's lanes; %.0f queries); lane work "
                        "(visits + steps) group max %.2f, wave max %.2f\n",
                        a / n, b / n, c / n, n, gm / n, wm / n);
            }
#endif
            fprintf(stderr,
                    "[orbx seq stamps] pairs=%d | grid %.1f, scoring %.1f us | commit mean/max %.1f/%.1f us | %.1f "
                    "queries, %.1f re-scored, replay iterations mean/max %.1f/%.0f | chunk loads %.1f, rounds %.1f, "
                    "commits %.1f, re-scoring %.1f us, %.1f stops\n",
                    npairs, gr / npairs, sc / npairs, cm / npairs, cmx, nq / npairs, resc / npairs, nit / npairs, itmx,
                    tl / npairs, tr / npairs, tcm / npairs, trs / npairs, nst / npairs);
            return ORBX_OK;
        }
        double ph[4] = {0, 0, 0, 0}, mx[4] = {0, 0, 0, 0}, resc = 0, nq = 0, nit = 0, tres = 0, tfirst = 0;
        double tbit = 0, tfill = 0, tbuild = 0, rtrunc = 0;
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int p = 0; p < npairs; p++) {
            const unsigned long long* r = &h[(size_t)kStampWords * p];
            tres += (double)r[8] * 0.01;
            tfirst += (double)r[9] * 0.01;
            for (int k = 0; k < 4; k++) {
                const double d = (double)(r[k + 1] - r[k]) * 0.01;  // 100 MHz -> us
                ph[k] += d;
                if (d > mx[k]) mx[k] = d;
            }
            resc += (double)r[5];
            rtrunc += (double)r[12];
            nq += (double)r[6];
            nit += (double)r[7];
            tbit += (double)(r[10] - r[0]) * 0.01;
            tfill += (double)(r[11] - r[10]) * 0.01;
            tbuild += (double)(r[1] - r[11]) * 0.01;
            if (r[0] < t0) t0 = r[0];
            if (r[4] > t1) t1 = r[4];
        }
        fprintf(stderr,
                "[orbx stamps] pairs=%d span=%.1fus | mean/max us: sort %.1f/%.1f score %.1f/%.1f commit %.1f/%.1f "
                "store %.1f/%.1f | rescored %.1f of %.1f queries (%.1f us), %.1f replay rounds (chunk loads + first "
                "rounds %.1f us) | sort = grid counting sort %.1f + column starts %.1f + octave runs and fill %.1f us | re-scored at a "
                "truncation %.1f\n",
                npairs, (double)(t1 - t0) * 0.01, ph[0] / npairs, mx[0], ph[1] / npairs, mx[1], ph[2] / npairs, mx[2],
                ph[3] / npairs, mx[3], resc / npairs, nq / npairs, tres / npairs, nit / npairs, tfirst / npairs,
                tbit / npairs, tfill / npairs, tbuild / npairs, rtrunc / npairs);
    }
    return ORBX_OK;
}

// Tracking::SearchLocalPoints for a batch of Frames in HBM (see include/orbx.h)
int orbx_search_local_points_device(orbx_matcher* m, const orbx_mappoints_device* mps,
                                    const orbx_local_map_batch* lm, void* stream) {
    if (!m || !mps || !lm) return fail(ORBX_ERR_ARG, "null argument");
    const int B = lm->batch, cap = lm->cap, nlevels = lm->nlevels;
    if (B < 0 || cap <= 0 || cap >= 8192 || !lm->scale_factors || nlevels < 2 || nlevels > 32 || !lm->local_off)
        return fail(ORBX_ERR_ARG, "bad argument");
    if (B == 0) return ORBX_OK;
    if (!lm->kps || !lm->desc || !lm->n || !lm->Tcw || !lm->frame_mp || !lm->nmatches || !mps->pos || !mps->desc ||
        !mps->normal || !mps->max_distance || !mps->min_distance || !mps->observations)
        return fail(ORBX_ERR_ARG, "null buffer");
    if (mps->n < 0 || mps->n >= kMaxMapPointIds) return fail(ORBX_ERR_ARG, "MapPoint table of 2^30 or more");
    int maxnq = 0;
    for (int b = 0; b < B; b++) {
        const int c = lm->local_off[b + 1] - lm->local_off[b];
        if (lm->local_off[b] < 0 || c < 0) return fail(ORBX_ERR_ARG, "local_off must be non-decreasing from 0");
        if (c > maxnq) maxnq = c;
    }
    const int total = lm->local_off[B];
    if (maxnq > (1 << 20)) return fail(ORBX_ERR_ARG, "a local map of more than 2^20 MapPoints");
    if (total > 0 && !lm->local_ids) return fail(ORBX_ERR_ARG, "null local_ids");
    // grids hold a frame's keypoints (cap < 8192, 13-bit sorted positions); the queries
    // (local MapPoints) are not position-encoded, so a local map may exceed that
    HIP_TRY(hipSetDevice(m->device));
    hipStream_t s = stream ? (hipStream_t)stream : m->stream;
    const bool split = m->footprint == 2;
    const bool grids = split || m->footprint == 5;
    const size_t nt = (size_t)(total > 0 ? total : 1);
    const size_t need = pad(sizeof(ProjQuery) * nt) + pad(nt * 32) + pad(sizeof(ProjProblem) * B) +
                        pad(sizeof(long long) * B) + pad(sizeof(unsigned long long) * kProjScratchWords * nt) +
                        pad(sizeof(int32_t) * (B + 1)) + (grids ? pad(seq_grid_bytes(cap, nlevels) * B) : 0);
    if (m->lscr_cap < need) {
        HIP_TRY(hipStreamSynchronize(s));
        if (m->lscr) HIP_TRY(hipFree(m->lscr));
        m->lscr = nullptr;
        m->lscr_cap = 0;
        HIP_TRY(hipMalloc((void**)&m->lscr, need));
        m->lscr_cap = need;
    }
    size_t o = 0;
    auto take = [&](size_t bytes) {
        char* p = m->lscr + o;
        o += pad(bytes);
        return p;
    };
    auto* d_q = (ProjQuery*)take(sizeof(ProjQuery) * nt);
    auto* d_qd = (uint8_t*)take(nt * 32);
    auto* d_prob = (ProjProblem*)take(sizeof(ProjProblem) * B);
    auto* d_off = (long long*)take(sizeof(long long) * B);
    auto* d_scr = (unsigned long long*)take(sizeof(unsigned long long) * kProjScratchWords * nt);
    auto* d_loff = (int32_t*)take(sizeof(int32_t) * (B + 1));
    auto* d_grids = grids ? (unsigned char*)take(seq_grid_bytes(cap, nlevels) * B) : nullptr;
    char* h = nullptr;
    int slot = 0;
    HIP_TRY(m->stage.get(sizeof(int32_t) * (B + 1), &h, &slot));
    std::memcpy(h, lm->local_off, sizeof(int32_t) * (B + 1));
    HIP_TRY(hipMemcpyAsync(d_loff, h, sizeof(int32_t) * (B + 1), hipMemcpyHostToDevice, s));
    HIP_TRY(m->stage.copied(slot, s));
    LocalArgs A{};
    A.kps = lm->kps;
    A.desc = lm->desc;
    A.n = lm->n;
    A.u_right = lm->u_right;
    A.cap = cap;
    A.Tcw = lm->Tcw;
    A.fx = lm->fx;
    A.fy = lm->fy;
    A.cx = lm->cx;
    A.cy = lm->cy;
    A.bf = lm->bf;
    A.min_x = lm->min_x;
    A.max_x = lm->max_x;
    A.min_y = lm->min_y;
    A.max_y = lm->max_y;
    for (int l = 0; l < nlevels; l++) A.scale[l] = lm->scale_factors[l];
    A.nlevels = nlevels;
    A.log_scale = (float)std::log((double)lm->scale_factors[1]);  // Frame::mfLogScaleFactor
    A.nmp = mps->n;
    A.pos = mps->pos;
    A.mdesc = mps->desc;
    A.normal = mps->normal;
    A.max_distance = mps->max_distance;
    A.min_distance = mps->min_distance;
    A.bad = mps->bad;
    A.local_off = d_loff;
    A.local_ids = lm->local_ids;
    A.th = lm->th;
    A.cos_limit = lm->viewing_cos_limit;
    A.frame_mp = lm->frame_mp;
    A.nmatches = lm->nmatches;
    int hs = 256;
    while (hs < 2 * cap) hs <<= 1;
    A.hash_size = hs;
    HIP_TRY(launch_local_build(A, B, d_q, d_qd, d_prob, d_off, s));
    ProjParams P{};
    P.mp_obs = mps->observations;
    P.blocked_mode = 0;  // a keypoint whose MapPoint has Observations() > 0 is taken (ORBmatcher.cc:117-119)
    P.accept_th = TH_HIGH;
    P.ratio_mode = 1;
    P.nnratio = m->nnratio;
    P.check_ori = 0;
    P.noct = nlevels;
    if (split)
        HIP_TRY(launch_seq_split(d_prob, B, P, d_grids, cap, d_scr, d_off, s, maxnq > 0 ? maxnq : 1));
    else
        HIP_TRY(launch_proj_search(d_prob, B, P, d_scr, d_off, cap, maxnq, s, m->footprint == 1, m->footprint == 3,
                                   m->footprint == 4, m->footprint == 5 ? d_grids : nullptr));
    return ORBX_OK;
}

int orbx_matcher_set_footprint(orbx_matcher* m, int small) {
    if (!m) return fail(ORBX_ERR_ARG, "null matcher");
    if (small < 0 || small > 5) return fail(ORBX_ERR_ARG, "footprint is 0 .. 5");
    m->footprint = small;
    return ORBX_OK;
}

int orbx_matcher_set_timing(orbx_matcher* m, int enable) {
    if (!m) return fail(ORBX_ERR_ARG, "null matcher");
    m->timing = enable != 0;
    m->ncalls = 0;
    return ORBX_OK;
}

double orbx_matcher_last_call_us(const orbx_matcher* m) { return m ? m->last_call_us : -1.0; }

int orbx_matcher_last_ms(orbx_matcher* m, float* ms) {
    if (!m || !ms) return fail(ORBX_ERR_ARG, "null argument");
    if (m->ncalls == 0) return fail(ORBX_ERR_STATE, "no timed call");
    const long long last = m->ncalls - 1;
    const int nslots = m->ncalls < orbx_matcher::kRing ? (int)m->ncalls : orbx_matcher::kRing;
    HIP_TRY(hipEventSynchronize(m->ev[last % orbx_matcher::kRing][1]));
    double sum = 0.0;
    for (int k = 0; k < nslots; k++) {
        hipEvent_t* e = m->ev[(last - k) % orbx_matcher::kRing];
        float t = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, e[0], e[1]));
        sum += t;
    }
    *ms = (float)(sum / nslots);
    return ORBX_OK;
}

// ORBmatcher::SearchForTriangulation, ORBmatcher.cc:850-1056
int orbx_search_for_triangulation(orbx_matcher* m, const orbx_frame_view* kf1, const uint8_t* kf1_has_mp,
                                  const int32_t* fv1_node, const int32_t* fv1_off, const int32_t* fv1_idx, int fv1_n,
                                  const orbx_frame_view* kf2, const uint8_t* kf2_has_mp, const int32_t* fv2_node,
                                  const int32_t* fv2_off, const int32_t* fv2_idx, int fv2_n, const float* F12,
                                  int only_stereo, int32_t* pairs, int* npairs) {
    const CallClock clock_(m);
    if (!m || !kf1 || !kf2 || !kf1_has_mp || !kf2_has_mp || !F12 || !pairs || !npairs)
        return fail(ORBX_ERR_ARG, "null argument");
    // epipole of KF1's centre in KF2 (cc:858-865)
    float Cw[3], C2[3];
    centre(kf1->Tcw, Cw);
    project(kf2->Tcw, Cw, C2);
    const float invz = 1.0f / C2[2];
    const float ex = std::fma(kf2->fx * C2[0], invz, kf2->cx);  // fused (H4)
    const float ey = std::fma(kf2->fy * C2[1], invz, kf2->cy);
    // queries in the reference's visiting order: shared nodes ascending (cc:886-1019)
    std::vector<TriQuery> qs;
    int f1 = 0, f2 = 0;
    while (f1 < fv1_n && f2 < fv2_n) {
        if (fv1_node[f1] == fv2_node[f2]) {
            for (int i1 = fv1_off[f1]; i1 < fv1_off[f1 + 1]; i1++) {
                const int idx1 = fv1_idx[i1];
                if (idx1 < 0 || idx1 >= kf1->n) return fail(ORBX_ERR_ARG, "feature index out of range");
                if (kf1_has_mp[idx1]) continue;
                const bool bStereo1 = kf1->u_right && kf1->u_right[idx1] >= 0;
                if (only_stereo && !bStereo1) continue;
                TriQuery q;
                q.idx1 = idx1;
                q.beg = fv2_off[f2];
                q.end = fv2_off[f2 + 1];
                q.stereo1 = bStereo1 ? 1 : 0;
                qs.push_back(q);
            }
            f1++;
            f2++;
        } else if (fv1_node[f1] < fv2_node[f2]) {
            f1 = (int)(std::lower_bound(fv1_node + f1, fv1_node + fv1_n, fv2_node[f2]) - fv1_node);
        } else {
            f2 = (int)(std::lower_bound(fv2_node + f2, fv2_node + fv2_n, fv1_node[f1]) - fv2_node);
        }
    }
    *npairs = 0;
    if (qs.empty()) return ORBX_OK;
    HIP_TRY(hipSetDevice(m->device));
    const int n1 = kf1->n, n2 = kf2->n, nq = (int)qs.size();
    const int nfv2 = fv2_off[fv2_n];
    const size_t need = pad(sizeof(orbx_keypoint) * n1) + pad((size_t)n1 * 32) + pad(sizeof(orbx_keypoint) * n2) +
                        pad((size_t)n2 * 32) + pad(sizeof(float) * n2) + pad(n2) + pad(sizeof(int32_t) * nfv2) +
                        2 * pad(sizeof(float) * 32) + pad(sizeof(TriQuery) * nq) + pad(sizeof(int32_t) * n1) +
                        pad(sizeof(TriProblem)) + pad(8 * (size_t)nq);
    HIP_TRY(m->arena.reserve(need));
    m->arena.used = 0;
    auto* d_k1 = m->arena.take<orbx_keypoint>(n1);
    auto* d_d1 = m->arena.take<uint8_t>((size_t)n1 * 32);
    auto* d_k2 = m->arena.take<orbx_keypoint>(n2);
    auto* d_d2 = m->arena.take<uint8_t>((size_t)n2 * 32);
    auto* d_ur2 = m->arena.take<float>(n2);
    auto* d_mp2 = m->arena.take<uint8_t>(n2);
    auto* d_fv2 = m->arena.take<int32_t>(nfv2);
    auto* d_sc2 = m->arena.take<float>(32);
    auto* d_sg2 = m->arena.take<float>(32);
    auto* d_q = m->arena.take<TriQuery>(nq);
    auto* d_m12 = m->arena.take<int32_t>(n1);
    auto* d_prob = m->arena.take<TriProblem>(1);
    auto* d_scr = m->arena.take<unsigned long long>(nq);
    hipStream_t s = m->stream;
    m->arena.up(d_k1, kf1->keys, sizeof(orbx_keypoint) * n1);
    m->arena.up(d_d1, kf1->desc, (size_t)n1 * 32);
    m->arena.up(d_k2, kf2->keys, sizeof(orbx_keypoint) * n2);
    m->arena.up(d_d2, kf2->desc, (size_t)n2 * 32);
    if (kf2->u_right) m->arena.up(d_ur2, kf2->u_right, sizeof(float) * n2);
    m->arena.up(d_mp2, kf2_has_mp, n2);
    if (nfv2) m->arena.up(d_fv2, fv2_idx, sizeof(int32_t) * nfv2);
    m->arena.up(d_sc2, kf2->scale_factors, sizeof(float) * kf2->nlevels);
    m->arena.up(d_sg2, kf2->level_sigma2, sizeof(float) * kf2->nlevels);
    m->arena.up(d_q, qs.data(), sizeof(TriQuery) * nq);
    m->arena.fill(d_m12, 0xff, sizeof(int32_t) * n1);
    TriProblem pb{};
    pb.keys1 = d_k1;
    pb.desc1 = d_d1;
    pb.keys2 = d_k2;
    pb.desc2 = d_d2;
    pb.u_right2 = kf2->u_right ? d_ur2 : nullptr;
    pb.has_mp2 = d_mp2;
    pb.fv2_idx = d_fv2;
    pb.scale2 = d_sc2;
    pb.sigma2_2 = d_sg2;
    std::memcpy(pb.F12, F12, sizeof(pb.F12));
    pb.ex = ex;
    pb.ey = ey;
    pb.only_stereo = only_stereo ? 1 : 0;
    pb.check_ori = m->check_ori;
    pb.n2 = n2;
    pb.q = d_q;
    pb.nq = nq;
    pb.matches12 = d_m12;
    pb.scratch_off = 0;
    m->arena.up(d_prob, &pb, sizeof(pb));
    HIP_TRY(m->arena.flush(s));
    HIP_TRY(launch_triangulation(d_prob, 1, d_scr, n2, nq, s));
    std::vector<int32_t> m12((size_t)n1);
    HIP_TRY(m->arena.down(m12.data(), d_m12, sizeof(int32_t) * n1, s));
    HIP_TRY(m->arena.sync(s));
    int np = 0;
    for (int i = 0; i < n1; i++) {  // vMatchedPairs in idx1 order (cc:1045-1053)
        if (m12[(size_t)i] < 0) continue;
        pairs[2 * np] = i;
        pairs[2 * np + 1] = m12[(size_t)i];
        np++;
    }
    *npairs = np;
    return ORBX_OK;
}

// LocalMapping::CreateNewMapPoints' SearchForTriangulation loop (LocalMapping.cc:235-305)
// over keyframes in HBM: the host part of ORBmatcher.cc:850-1056 (the epipole, cc:858-865)
// per pair here, the FeatureVector merge and the scoring / commit on the device.
int orbx_search_for_triangulation_batch_device(orbx_matcher* m, int nkf, const orbx_keyframe_device* kfs,
                                               const orbx_frame_view* cam, int npairs, const int32_t* pairs,
                                               const float* F12, int only_stereo, int cap, int32_t* d_matches12,
                                               int32_t* d_pairs, int32_t* d_npairs, void* stream) {
    if (!m || nkf < 0 || npairs < 0 || !cam) return fail(ORBX_ERR_ARG, "bad argument");
    if (npairs == 0) return ORBX_OK;
    if (!kfs || !pairs || !F12 || !d_matches12 || !d_pairs || !d_npairs) return fail(ORBX_ERR_ARG, "null buffer");
    if (cap <= 0) return fail(ORBX_ERR_ARG, "bad cap");
    if (cap > 8192) return fail(ORBX_ERR_UNSUPPORTED, "cap above 8192 keypoints per keyframe");
    if (cam->nlevels < 1 || cam->nlevels > ORBX_MAX_LEVELS || !cam->scale_factors || !cam->level_sigma2)
        return fail(ORBX_ERR_ARG, "bad level tables");
    for (int k = 0; k < nkf; k++) {
        const orbx_keyframe_device& K = kfs[k];
        if (!K.keys || !K.desc || !K.n || !K.has_mp || !K.fv_node || !K.fv_off || !K.fv_idx || !K.nfv)
            return fail(ORBX_ERR_ARG, "null keyframe array");
    }
    std::vector<TriKF> tk((size_t)nkf);
    for (int k = 0; k < nkf; k++) {
        const orbx_keyframe_device& K = kfs[k];
        tk[(size_t)k] = TriKF{K.keys, K.desc, K.n, K.u_right, K.has_mp, K.fv_node, K.fv_off, K.fv_idx, K.nfv};
    }
    std::vector<TriPair> tp((size_t)npairs);
    for (int p = 0; p < npairs; p++) {
        const int a = pairs[2 * p], b = pairs[2 * p + 1];
        if (a < 0 || a >= nkf || b < 0 || b >= nkf) return fail(ORBX_ERR_ARG, "keyframe index out of range");
        TriPair& t = tp[(size_t)p];
        t.kf1 = a;
        t.kf2 = b;
        std::memcpy(t.F12, F12 + 9 * (size_t)p, sizeof(t.F12));
        // epipole of KF1's centre in KF2 (cc:858-865), as orbx_search_for_triangulation
        float Cw[3], C2[3];
        centre(kfs[a].Tcw, Cw);
        project(kfs[b].Tcw, Cw, C2);
        const float invz = 1.0f / C2[2];
        t.ex = std::fma(cam->fx * C2[0], invz, cam->cx);  // fused (H4)
        t.ey = std::fma(cam->fy * C2[1], invz, cam->cy);
    }
    HIP_TRY(hipSetDevice(m->device));
    hipStream_t s = stream ? (hipStream_t)stream : m->stream;
    const size_t P = (size_t)npairs;
    const size_t need = pad(sizeof(TriKF) * (size_t)nkf) + pad(sizeof(TriPair) * P) + 2 * pad(sizeof(float) * 32) +
                        pad(sizeof(TriQuery) * P * cap) + pad(sizeof(TriProblem) * P) +
                        pad(sizeof(unsigned long long) * P * cap);
    if (m->tscr_cap < need) {
        HIP_TRY(hipStreamSynchronize(s));
        if (m->tscr) HIP_TRY(hipFree(m->tscr));
        m->tscr = nullptr;
        m->tscr_cap = 0;
        HIP_TRY(hipMalloc((void**)&m->tscr, need));
        m->tscr_cap = need;
    }
    // tables first (one staged copy), then the device-only work areas
    const size_t tab = pad(sizeof(TriKF) * (size_t)nkf) + pad(sizeof(TriPair) * P) + 2 * pad(sizeof(float) * 32);
    char* q = m->tscr;
    auto take = [&q](size_t bytes) {
        char* r = q;
        q += pad(bytes);
        return r;
    };
    TriBatch tb{};
    auto* d_kf = (TriKF*)take(sizeof(TriKF) * (size_t)nkf);
    auto* d_tp = (TriPair*)take(sizeof(TriPair) * P);
    auto* d_sc = (float*)take(sizeof(float) * 32);
    auto* d_sg = (float*)take(sizeof(float) * 32);
    tb.q = (TriQuery*)take(sizeof(TriQuery) * P * cap);
    tb.probs = (TriProblem*)take(sizeof(TriProblem) * P);
    auto* d_scr = (unsigned long long*)take(sizeof(unsigned long long) * P * cap);
    char* h = nullptr;
    int slot = 0;
    HIP_TRY(m->stage.get(tab, &h, &slot));
    std::memset(h, 0, tab);
    std::memcpy(h + ((char*)d_kf - m->tscr), tk.data(), sizeof(TriKF) * (size_t)nkf);
    std::memcpy(h + ((char*)d_tp - m->tscr), tp.data(), sizeof(TriPair) * P);
    float* hs = (float*)(h + ((char*)d_sc - m->tscr));
    float* hg = (float*)(h + ((char*)d_sg - m->tscr));
    for (int l = 0; l < cam->nlevels; l++) {
        hs[l] = cam->scale_factors[l];
        hg[l] = cam->level_sigma2[l];
    }
    HIP_TRY(hipMemcpyAsync(m->tscr, h, tab, hipMemcpyHostToDevice, s));
    HIP_TRY(m->stage.copied(slot, s));
    tb.kfs = d_kf;
    tb.pairs = d_tp;
    tb.npairs = npairs;
    tb.cap = cap;
    tb.only_stereo = only_stereo ? 1 : 0;
    tb.check_ori = m->check_ori;
    tb.scale2 = d_sc;
    tb.sigma2_2 = d_sg;
    tb.matches12 = d_matches12;
    tb.pairs_out = d_pairs;
    tb.npairs_out = d_npairs;
    hipEvent_t* ev = m->ev[m->ncalls % orbx_matcher::kRing];
    if (m->timing) {
        for (int i = 0; i < 2; i++)
            if (!ev[i]) HIP_TRY(hipEventCreate(&ev[i]));
        HIP_TRY(hipEventRecord(ev[0], s));
    }
    HIP_TRY(launch_triangulation_batch(tb, d_scr, s));
    if (m->timing) {
        HIP_TRY(hipEventRecord(ev[1], s));
        m->ncalls++;
    }
    return ORBX_OK;
}

namespace {

// Shared vocabulary nodes in the reference's visiting order (ascending node id, the
// lower_bound walk of ORBmatcher.cc:254-358 / 721-814) with each node's side-1 queries.
int bow_nodes(const int32_t* fv1_node, const int32_t* fv1_off, const int32_t* fv1_idx, int fv1_n, int n1,
              const int32_t* fv2_node, const int32_t* fv2_off, int fv2_n, const int32_t* mp1,
              std::vector<BowNode>& nodes, std::vector<int32_t>& qidx) {
    int f1 = 0, f2 = 0;
    while (f1 < fv1_n && f2 < fv2_n) {
        if (fv1_node[f1] == fv2_node[f2]) {
            BowNode nd;
            nd.q_beg = (int)qidx.size();
            for (int i = fv1_off[f1]; i < fv1_off[f1 + 1]; i++) {
                const int idx1 = fv1_idx[i];
                if (idx1 < 0 || idx1 >= n1) return fail(ORBX_ERR_ARG, "feature index out of range");
                if (mp1[idx1] < 0) continue;  // !pMP || pMP->isBad()
                qidx.push_back(idx1);
            }
            nd.q_end = (int)qidx.size();
            nd.c_beg = fv2_off[f2];
            nd.c_end = fv2_off[f2 + 1];
            if (nd.c_end - nd.c_beg > 65535) return fail(ORBX_ERR_UNSUPPORTED, "vocabulary node with > 65535 features");
            if (nd.q_end > nd.q_beg && nd.c_end > nd.c_beg) nodes.push_back(nd);
            f1++;
            f2++;
        } else if (fv1_node[f1] < fv2_node[f2]) {
            f1 = (int)(std::lower_bound(fv1_node + f1, fv1_node + fv1_n, fv2_node[f2]) - fv1_node);
        } else {
            f2 = (int)(std::lower_bound(fv2_node + f2, fv2_node + fv2_n, fv1_node[f1]) - fv2_node);
        }
    }
    return ORBX_OK;
}

int run_bow(orbx_matcher* m, const orbx_frame_view* v1, const int32_t* mp1, const int32_t* fv1_node,
            const int32_t* fv1_off, const int32_t* fv1_idx, int fv1_n, const orbx_frame_view* v2, const int32_t* mp2,
            const int32_t* fv2_node, const int32_t* fv2_off, const int32_t* fv2_idx, int fv2_n, bool kf_kf,
            int32_t* matches, int* nmatches) {
    const int n1 = v1->n, n2 = v2->n, nout = kf_kf ? n1 : n2;
    for (int i = 0; i < nout; i++) matches[i] = -1;
    *nmatches = 0;
    std::vector<BowNode> nodes;
    std::vector<int32_t> qidx;
    int rc = bow_nodes(fv1_node, fv1_off, fv1_idx, fv1_n, n1, fv2_node, fv2_off, fv2_n, mp1, nodes, qidx);
    if (rc != ORBX_OK) return rc;
    if (nodes.empty()) return ORBX_OK;
    const int nfv2 = fv2_off[fv2_n];  // fv2_n > 0 here (a node is shared)
    for (int i = 0; i < nfv2; i++)
        if (fv2_idx[i] < 0 || fv2_idx[i] >= n2) return fail(ORBX_ERR_ARG, "feature index out of range");
    std::vector<uint8_t> avail;
    if (kf_kf) {  // vbMatched2 starts false; !pMP2 || pMP2->isBad() never match
        avail.resize((size_t)n2);
        for (int i = 0; i < n2; i++) avail[(size_t)i] = mp2[i] >= 0;
    }
    HIP_TRY(hipSetDevice(m->device));
    const int nq = (int)qidx.size(), nn = (int)nodes.size();
    const size_t need = pad(sizeof(orbx_keypoint) * n1) + pad((size_t)n1 * 32) + pad(sizeof(orbx_keypoint) * n2) +
                        pad((size_t)n2 * 32) + pad(sizeof(int32_t) * nq) + pad(sizeof(int32_t) * nfv2) + pad(n2) +
                        pad(sizeof(int32_t) * n1) + pad(sizeof(int32_t) * n2) + pad(sizeof(BowNode) * nn) +
                        pad(sizeof(int32_t) * nout) + pad(sizeof(BowProblem));
    HIP_TRY(m->arena.reserve(need));
    m->arena.used = 0;
    auto* d_k1 = m->arena.take<orbx_keypoint>(n1);
    auto* d_d1 = m->arena.take<uint8_t>((size_t)n1 * 32);
    auto* d_k2 = m->arena.take<orbx_keypoint>(n2);
    auto* d_d2 = m->arena.take<uint8_t>((size_t)n2 * 32);
    auto* d_q = m->arena.take<int32_t>(nq);
    auto* d_fv2 = m->arena.take<int32_t>(nfv2);
    auto* d_av = m->arena.take<uint8_t>(n2);
    auto* d_mp1 = m->arena.take<int32_t>(n1);
    auto* d_mp2 = m->arena.take<int32_t>(n2);
    auto* d_nodes = m->arena.take<BowNode>(nn);
    auto* d_out = m->arena.take<int32_t>(nout);
    auto* d_prob = m->arena.take<BowProblem>(1);
    hipStream_t s = m->stream;
    m->arena.up(d_k1, v1->keys, sizeof(orbx_keypoint) * n1);
    m->arena.up(d_d1, v1->desc, (size_t)n1 * 32);
    m->arena.up(d_k2, v2->keys, sizeof(orbx_keypoint) * n2);
    m->arena.up(d_d2, v2->desc, (size_t)n2 * 32);
    m->arena.up(d_q, qidx.data(), sizeof(int32_t) * nq);
    m->arena.up(d_fv2, fv2_idx, sizeof(int32_t) * nfv2);
    if (kf_kf) {
        m->arena.up(d_av, avail.data(), n2);
        m->arena.up(d_mp2, mp2, sizeof(int32_t) * n2);
    } else {
        m->arena.up(d_mp1, mp1, sizeof(int32_t) * n1);
    }
    m->arena.up(d_nodes, nodes.data(), sizeof(BowNode) * nn);
    m->arena.fill(d_out, 0xff, sizeof(int32_t) * nout);
    BowProblem pb{};
    pb.desc1 = d_d1;
    pb.keys1 = d_k1;
    pb.desc2 = d_d2;
    pb.keys2 = d_k2;
    pb.q_idx1 = d_q;
    pb.fv2_idx = d_fv2;
    pb.avail2 = kf_kf ? d_av : nullptr;
    pb.mp1 = d_mp1;
    pb.mp2 = d_mp2;
    pb.nodes = d_nodes;
    pb.nnodes = nn;
    pb.n1 = n1;
    pb.n2 = n2;
    pb.kf_kf = kf_kf ? 1 : 0;
    pb.nnratio = m->nnratio;
    pb.check_ori = m->check_ori;
    pb.matches = d_out;
    m->arena.up(d_prob, &pb, sizeof(pb));
    HIP_TRY(m->arena.flush(s));
    HIP_TRY(launch_bow(d_prob, n2, nout, s));
    HIP_TRY(m->arena.down(matches, d_out, sizeof(int32_t) * nout, s));
    HIP_TRY(m->arena.sync(s));
    int nm = 0;
    for (int i = 0; i < nout; i++) nm += matches[i] >= 0;
    *nmatches = nm;
    return ORBX_OK;
}

}  // namespace

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&), ORBmatcher.cc:228-392
int orbx_search_by_bow_frame(orbx_matcher* m, const orbx_frame_view* kf, const int32_t* kf_mp,
                             const int32_t* kf_fv_node, const int32_t* kf_fv_off, const int32_t* kf_fv_idx,
                             int kf_fv_n, const orbx_frame_view* f, const int32_t* f_fv_node, const int32_t* f_fv_off,
                             const int32_t* f_fv_idx, int f_fv_n, int32_t* matches, int* nmatches) {
    const CallClock clock_(m);
    if (!m || !kf || !f || !kf_mp || !matches || !nmatches || (kf_fv_n && (!kf_fv_node || !kf_fv_off || !kf_fv_idx)) ||
        (f_fv_n && (!f_fv_node || !f_fv_off || !f_fv_idx)) || kf_fv_n < 0 || f_fv_n < 0)
        return fail(ORBX_ERR_ARG, "null argument");
    return run_bow(m, kf, kf_mp, kf_fv_node, kf_fv_off, kf_fv_idx, kf_fv_n, f, nullptr, f_fv_node, f_fv_off, f_fv_idx,
                   f_fv_n, false, matches, nmatches);
}

// ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&), ORBmatcher.cc:696-839
int orbx_search_by_bow_keyframes(orbx_matcher* m, const orbx_frame_view* kf1, const int32_t* mp1,
                                 const int32_t* fv1_node, const int32_t* fv1_off, const int32_t* fv1_idx, int fv1_n,
                                 const orbx_frame_view* kf2, const int32_t* mp2, const int32_t* fv2_node,
                                 const int32_t* fv2_off, const int32_t* fv2_idx, int fv2_n, int32_t* matches12,
                                 int* nmatches) {
    const CallClock clock_(m);
    if (!m || !kf1 || !kf2 || !mp1 || !mp2 || !matches12 || !nmatches || (fv1_n && (!fv1_node || !fv1_off || !fv1_idx)) ||
        (fv2_n && (!fv2_node || !fv2_off || !fv2_idx)) || fv1_n < 0 || fv2_n < 0)
        return fail(ORBX_ERR_ARG, "null argument");
    return run_bow(m, kf1, mp1, fv1_node, fv1_off, fv1_idx, fv1_n, kf2, mp2, fv2_node, fv2_off, fv2_idx, fv2_n, true,
                   matches12, nmatches);
}

// ORBmatcher::SearchForInitialization, ORBmatcher.cc:539-683
int orbx_search_for_initialization(orbx_matcher* m, const orbx_frame_view* f1, const orbx_frame_view* f2,
                                   float* prev_matched, int32_t* matches12, int window_size, int* nmatches) {
    const CallClock clock_(m);
    if (!m || !f1 || !f2 || !prev_matched || !matches12 || !nmatches) return fail(ORBX_ERR_ARG, "null argument");
    const int n1 = f1->n, n2 = f2->n;
    if (n1 >= (1 << 20) || n2 >= (1 << 20)) return fail(ORBX_ERR_UNSUPPORTED, "more than 2^20 keypoints");
    for (int i = 0; i < n1; i++) matches12[i] = -1;
    *nmatches = 0;
    std::vector<int32_t> qidx;
    for (int i = 0; i < n1; i++)
        if (f1->keys[i].octave <= 0) qidx.push_back(i);  // level1 > 0 skipped (cc:562-564)
    // Frame::AssignFeaturesToGrid (Frame.cc:351-370) of F2 as CSR
    const float inv_w = (float)kGridCols / (f2->max_x - f2->min_x);
    const float inv_h = (float)kGridRows / (f2->max_y - f2->min_y);
    std::vector<int32_t> cstart(kNumCellsHost + 1, 0), cell((size_t)n2), cidx;
    for (int i = 0; i < n2; i++) {
        const int px = (int)roundf((f2->keys[i].x - f2->min_x) * inv_w);  // PosInGrid, Frame.cc:558-567
        const int py = (int)roundf((f2->keys[i].y - f2->min_y) * inv_h);
        cell[(size_t)i] = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : px * kGridRows + py;
        if (cell[(size_t)i] >= 0) cstart[cell[(size_t)i] + 1]++;
    }
    for (int c = 0; c < kNumCellsHost; c++) cstart[c + 1] += cstart[c];
    cidx.resize((size_t)cstart[kNumCellsHost] + 1);
    {
        std::vector<int32_t> fill(cstart.begin(), cstart.end() - 1);
        for (int i = 0; i < n2; i++)
            if (cell[(size_t)i] >= 0) cidx[(size_t)fill[cell[(size_t)i]]++] = i;
    }
    const int nq = (int)qidx.size();
    if (nq == 0 || n2 == 0) return ORBX_OK;
    const size_t lds = (size_t)4 * (2 * n2 + n1 + nq) + (size_t)nq + 16;
    if (lds > 160 * 1024) return fail(ORBX_ERR_UNSUPPORTED, "frames too large for one workgroup");
    HIP_TRY(hipSetDevice(m->device));
    const size_t need = pad(sizeof(orbx_keypoint) * n1) + pad((size_t)n1 * 32) + pad(sizeof(orbx_keypoint) * n2) +
                        pad((size_t)n2 * 32) + pad(sizeof(int32_t) * (kNumCellsHost + 1)) + pad(sizeof(int32_t) * cidx.size()) +
                        pad(sizeof(int32_t) * nq) + pad(sizeof(float) * 2 * n1) + pad(sizeof(int32_t) * n1) +
                        pad(8 * (size_t)nq * 8) + pad(sizeof(int) * nq) + pad(sizeof(InitProblem));
    HIP_TRY(m->arena.reserve(need));
    m->arena.used = 0;
    auto* d_k1 = m->arena.take<orbx_keypoint>(n1);
    auto* d_d1 = m->arena.take<uint8_t>((size_t)n1 * 32);
    auto* d_k2 = m->arena.take<orbx_keypoint>(n2);
    auto* d_d2 = m->arena.take<uint8_t>((size_t)n2 * 32);
    auto* d_cs = m->arena.take<int32_t>(kNumCellsHost + 1);
    auto* d_ci = m->arena.take<int32_t>(cidx.size());
    auto* d_q = m->arena.take<int32_t>(nq);
    auto* d_prev = m->arena.take<float>(2 * (size_t)n1);
    auto* d_m12 = m->arena.take<int32_t>(n1);
    auto* d_lists = m->arena.take<unsigned long long>((size_t)nq * 8);
    auto* d_tr = m->arena.take<int>(nq);
    auto* d_prob = m->arena.take<InitProblem>(1);
    hipStream_t s = m->stream;
    m->arena.up(d_k1, f1->keys, sizeof(orbx_keypoint) * n1);
    m->arena.up(d_d1, f1->desc, (size_t)n1 * 32);
    m->arena.up(d_k2, f2->keys, sizeof(orbx_keypoint) * n2);
    m->arena.up(d_d2, f2->desc, (size_t)n2 * 32);
    m->arena.up(d_cs, cstart.data(), sizeof(int32_t) * cstart.size());
    m->arena.up(d_ci, cidx.data(), sizeof(int32_t) * cidx.size());
    m->arena.up(d_q, qidx.data(), sizeof(int32_t) * nq);
    m->arena.up(d_prev, prev_matched, sizeof(float) * 2 * n1);
    InitProblem pb{};
    pb.keys1 = d_k1;
    pb.desc1 = d_d1;
    pb.keys2 = d_k2;
    pb.desc2 = d_d2;
    pb.cell_start = d_cs;
    pb.cell_idx = d_ci;
    pb.q_idx1 = d_q;
    pb.prev = d_prev;
    pb.nq = nq;
    pb.n1 = n1;
    pb.n2 = n2;
    pb.min_x = f2->min_x;
    pb.min_y = f2->min_y;
    pb.inv_w = inv_w;
    pb.inv_h = inv_h;
    pb.r = (float)window_size;
    pb.nnratio = m->nnratio;
    pb.check_ori = m->check_ori;
    pb.matches12 = d_m12;
    pb.lists = d_lists;
    pb.trunc = d_tr;
    m->arena.up(d_prob, &pb, sizeof(pb));
    HIP_TRY(m->arena.flush(s));
    HIP_TRY(launch_init(d_prob, n1, n2, nq, s));
    HIP_TRY(m->arena.down(matches12, d_m12, sizeof(int32_t) * n1, s));
    HIP_TRY(m->arena.sync(s));
    int nm = 0;
    for (int i = 0; i < n1; i++) {
        const int j = matches12[i];
        if (j < 0) continue;
        nm++;
        prev_matched[2 * i] = f2->keys[j].x;  // vbPrevMatched[i1] = F2.mvKeysUn[..].pt (cc:676-678)
        prev_matched[2 * i + 1] = f2->keys[j].y;
    }
    *nmatches = nm;
    return ORBX_OK;
}

namespace {

// Frame::AssignFeaturesToGrid (Frame.cc:351-370) of a view, as CSR (cell c = ix*ROWS + iy).
void host_grid(const orbx_frame_view* f, std::vector<int32_t>& cstart, std::vector<int32_t>& cidx, float& inv_w,
               float& inv_h) {
    inv_w = (float)kGridCols / (f->max_x - f->min_x);
    inv_h = (float)kGridRows / (f->max_y - f->min_y);
    cstart.assign(kNumCellsHost + 1, 0);
    std::vector<int32_t> cell((size_t)f->n);
    for (int i = 0; i < f->n; i++) {
        const int px = (int)roundf((f->keys[i].x - f->min_x) * inv_w);  // PosInGrid, Frame.cc:558-567
        const int py = (int)roundf((f->keys[i].y - f->min_y) * inv_h);
        cell[(size_t)i] = (px < 0 || px >= kGridCols || py < 0 || py >= kGridRows) ? -1 : px * kGridRows + py;
        if (cell[(size_t)i] >= 0) cstart[cell[(size_t)i] + 1]++;
    }
    for (int c = 0; c < kNumCellsHost; c++) cstart[c + 1] += cstart[c];
    cidx.assign((size_t)cstart[kNumCellsHost] + 1, 0);
    std::vector<int32_t> fill(cstart.begin(), cstart.end() - 1);
    for (int i = 0; i < f->n; i++)
        if (cell[(size_t)i] >= 0) cidx[(size_t)fill[cell[(size_t)i]]++] = i;
}

// Window-best search of `qs` in keyframe `f` (one k_window_best launch); best[k] out.
int run_best(orbx_matcher* m, const orbx_frame_view* f, const std::vector<BestQuery>& qs,
             const std::vector<uint8_t>& qd, int gate, int accept, int32_t* best) {
    const int nq = (int)qs.size(), n = f->n;
    if (nq == 0) return ORBX_OK;
    if (n == 0) {
        for (int k = 0; k < nq; k++) best[k] = -1;
        return ORBX_OK;
    }
    std::vector<int32_t> cstart, cidx;
    float inv_w, inv_h;
    host_grid(f, cstart, cidx, inv_w, inv_h);
    HIP_TRY(hipSetDevice(m->device));
    const size_t need = pad(sizeof(orbx_keypoint) * n) + pad((size_t)n * 32) + pad(sizeof(float) * n) +
                        pad(sizeof(int32_t) * cstart.size()) + pad(sizeof(int32_t) * cidx.size()) +
                        pad(sizeof(BestQuery) * nq) + pad((size_t)nq * 32) + pad(sizeof(int32_t) * nq) +
                        pad(sizeof(BestProblem));
    HIP_TRY(m->arena.reserve(need));
    m->arena.used = 0;
    auto* d_k = m->arena.take<orbx_keypoint>(n);
    auto* d_d = m->arena.take<uint8_t>((size_t)n * 32);
    auto* d_ur = m->arena.take<float>(n);
    auto* d_cs = m->arena.take<int32_t>(cstart.size());
    auto* d_ci = m->arena.take<int32_t>(cidx.size());
    auto* d_q = m->arena.take<BestQuery>(nq);
    auto* d_qd = m->arena.take<uint8_t>((size_t)nq * 32);
    auto* d_best = m->arena.take<int32_t>(nq);
    auto* d_prob = m->arena.take<BestProblem>(1);
    hipStream_t s = m->stream;
    m->arena.up(d_k, f->keys, sizeof(orbx_keypoint) * n);
    m->arena.up(d_d, f->desc, (size_t)n * 32);
    if (gate && f->u_right) m->arena.up(d_ur, f->u_right, sizeof(float) * n);
    m->arena.up(d_cs, cstart.data(), sizeof(int32_t) * cstart.size());
    m->arena.up(d_ci, cidx.data(), sizeof(int32_t) * cidx.size());
    m->arena.up(d_q, qs.data(), sizeof(BestQuery) * nq);
    m->arena.up(d_qd, qd.data(), (size_t)nq * 32);
    BestProblem pb{};
    pb.keys = d_k;
    pb.desc = d_d;
    pb.u_right = (gate && f->u_right) ? d_ur : nullptr;
    pb.cell_start = d_cs;
    pb.cell_idx = d_ci;
    for (int l = 0; l < f->nlevels && l < 32; l++) pb.inv_sigma2[l] = 1.0f / f->level_sigma2[l];  // mvInvLevelSigma2
    pb.min_x = f->min_x;
    pb.min_y = f->min_y;
    pb.inv_w = inv_w;
    pb.inv_h = inv_h;
    pb.q = d_q;
    pb.qdesc = d_qd;
    pb.nq = nq;
    pb.gate = gate;
    pb.accept = accept;
    pb.best = d_best;
    m->arena.up(d_prob, &pb, sizeof(pb));
    HIP_TRY(m->arena.flush(s));
    HIP_TRY(launch_window_best(d_prob, nq, s));
    HIP_TRY(m->arena.down(best, d_best, sizeof(int32_t) * nq, s));
    HIP_TRY(m->arena.sync(s));
    return ORBX_OK;
}

bool in_image(const orbx_frame_view* f, float u, float v) {  // KeyFrame::IsInImage, KeyFrame.cc:661-663
    return u >= f->min_x && u < f->max_x && v >= f->min_y && v < f->max_y;
}

// Shared tail of both Fuse overloads: distance / viewing-angle checks, PredictScale,
// query record.  Returns false when the MapPoint is rejected before the window search.
bool fuse_query(const orbx_frame_view* kf, const orbx_mappoints* mps, int mp, const float* Ow, float u, float v,
                float ur, float th, BestQuery& q) {
    const float* p3Dw = mps->pos + 3 * (size_t)mp;
    float PO[3];
    for (int c = 0; c < 3; c++) PO[c] = p3Dw[c] - Ow[c];
    const float dist3D = norm3(PO);
    if (dist3D < 0.8f * mps->min_distance[mp] || dist3D > 1.2f * mps->max_distance[mp]) return false;
    const float* Pn = mps->normal + 3 * (size_t)mp;
    double dot = 0.0;  // Mat::dot accumulates in double
    for (int c = 0; c < 3; c++) dot += (double)PO[c] * Pn[c];
    if (dot < 0.5 * dist3D) return false;
    const int pred = predict_scale(mps->max_distance[mp], dist3D, kf);
    q = BestQuery{};
    q.u = u;
    q.v = v;
    q.ur = ur;
    q.r = th * kf->scale_factors[pred];
    q.pred = pred;
    return true;
}

bool mps_ok(const orbx_mappoints* mps, bool need_normal) {
    return mps && mps->pos && mps->desc && mps->max_distance && mps->min_distance && (!need_normal || mps->normal);
}

}  // namespace

// ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, th), ORBmatcher.cc:1067-1221
int orbx_fuse(orbx_matcher* m, const orbx_frame_view* kf, const int32_t* points, int npoints, const uint8_t* skip,
              const orbx_mappoints* mps, float th, int32_t* best) {
    const CallClock clock_(m);
    if (!m || !kf || !skip || !best || !mps_ok(mps, true) || npoints < 0 || (npoints && !points))
        return fail(ORBX_ERR_ARG, "null argument");
    if (kf->nlevels < 2) return fail(ORBX_ERR_ARG, "need >= 2 pyramid levels");
    float Ow[3];
    centre(kf->Tcw, Ow);
    std::vector<BestQuery> qs;
    std::vector<uint8_t> qd;
    std::vector<int> slot;
    for (int k = 0; k < npoints; k++) {
        best[k] = -1;
        const int mp = points[k];
        if (mp < 0) continue;
        if (mp >= mps->n) return fail(ORBX_ERR_ARG, "MapPoint id out of range");
        if (skip[mp]) continue;  // isBad() || IsInKeyFrame(pKF)
        float p3Dc[3];
        project(kf->Tcw, mps->pos + 3 * (size_t)mp, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = 1 / p3Dc[2];
        const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
        const float u = std::fma(kf->fx, x, kf->cx), v = std::fma(kf->fy, y, kf->cy);  // fused (H4)
        if (!in_image(kf, u, v)) continue;
        const float ur = std::fma(-kf->bf, invz, u);
        BestQuery q;
        if (!fuse_query(kf, mps, mp, Ow, u, v, ur, th, q)) continue;
        qs.push_back(q);
        qd.insert(qd.end(), mps->desc + (size_t)mp * 32, mps->desc + (size_t)mp * 32 + 32);
        slot.push_back(k);
    }
    std::vector<int32_t> out(qs.size());
    const int rc = run_best(m, kf, qs, qd, 1, TH_LOW, out.data());
    if (rc != ORBX_OK) return rc;
    for (size_t j = 0; j < slot.size(); j++) best[slot[j]] = out[j];
    return ORBX_OK;
}

// ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, const vector<MapPoint*>& vpPoints, th,
// vector<MapPoint*>& vpReplacePoint), ORBmatcher.cc:1226-1352
int orbx_fuse_sim3(orbx_matcher* m, const orbx_frame_view* kf, const float* Scw, const int32_t* points, int npoints,
                   const uint8_t* skip, const orbx_mappoints* mps, float th, int32_t* best) {
    const CallClock clock_(m);
    if (!m || !kf || !Scw || !skip || !best || !mps_ok(mps, true) || npoints < 0 || (npoints && !points))
        return fail(ORBX_ERR_ARG, "null argument");
    if (kf->nlevels < 2) return fail(ORBX_ERR_ARG, "need >= 2 pyramid levels");
    double d0 = 0.0;
    for (int c = 0; c < 3; c++) d0 += (double)Scw[c] * Scw[c];
    const float scw = (float)std::sqrt(d0);  // cc:1234
    const float alpha = (float)(1.0 / scw);
    float T[12];
    for (int k = 0; k < 12; k++) T[k] = Scw[k] * alpha;
    float Ow[3];
    centre(T, Ow);
    std::vector<BestQuery> qs;
    std::vector<uint8_t> qd;
    std::vector<int> slot;
    for (int k = 0; k < npoints; k++) {
        best[k] = -1;
        const int mp = points[k];
        if (mp < 0 || mp >= mps->n) return fail(ORBX_ERR_ARG, "MapPoint id out of range");
        if (skip[mp]) continue;  // isBad() || spAlreadyFound.count(pMP)
        float p3Dc[3];
        project(T, mps->pos + 3 * (size_t)mp, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = (float)(1.0 / p3Dc[2]);
        const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
        const float u = std::fma(kf->fx, x, kf->cx), v = std::fma(kf->fy, y, kf->cy);  // fused (H4)
        if (!in_image(kf, u, v)) continue;
        BestQuery q;
        if (!fuse_query(kf, mps, mp, Ow, u, v, 0.f, th, q)) continue;
        qs.push_back(q);
        qd.insert(qd.end(), mps->desc + (size_t)mp * 32, mps->desc + (size_t)mp * 32 + 32);
        slot.push_back(k);
    }
    std::vector<int32_t> out(qs.size());
    const int rc = run_best(m, kf, qs, qd, 0, TH_LOW, out.data());
    if (rc != ORBX_OK) return rc;
    for (size_t j = 0; j < slot.size(); j++) best[slot[j]] = out[j];
    return ORBX_OK;
}

namespace {

// One direction of SearchBySim3 (cc:1408-1475 / 1477-1545): MapPoints of `src` mapped by
// x_dst = sR (R_src x + t_src) + t into `dst`, window-searched there (accept <= TH_HIGH).
int sim3_direction(orbx_matcher* m, const orbx_frame_view* src, const int32_t* src_mp, const uint8_t* already,
                   const orbx_frame_view* dst, const orbx_mappoints* mps, const float* sR, const float* t, float th,
                   std::vector<int32_t>& vnMatch) {
    vnMatch.assign((size_t)src->n, -1);
    std::vector<BestQuery> qs;
    std::vector<uint8_t> qd;
    std::vector<int> slot;
    for (int i = 0; i < src->n; i++) {
        const int mp = src_mp[i];
        if (mp < 0 || (already && already[i])) continue;
        if (mp >= mps->n) return fail(ORBX_ERR_ARG, "MapPoint id out of range");
        if (mps->bad && mps->bad[mp]) continue;
        float pc[3], pd[3];
        project(src->Tcw, mps->pos + 3 * (size_t)mp, pc);
        for (int r = 0; r < 3; r++) pd[r] = sR[3 * r] * pc[0] + sR[3 * r + 1] * pc[1] + sR[3 * r + 2] * pc[2] + t[r];
        if (pd[2] < 0.0) continue;
        const float invz = (float)(1.0 / pd[2]);
        const float x = pd[0] * invz, y = pd[1] * invz;
        const float u = std::fma(dst->fx, x, dst->cx), v = std::fma(dst->fy, y, dst->cy);  // fused (H4)
        if (!in_image(dst, u, v)) continue;
        const float dist3D = norm3(pd);
        if (dist3D < 0.8f * mps->min_distance[mp] || dist3D > 1.2f * mps->max_distance[mp]) continue;
        const int pred = predict_scale(mps->max_distance[mp], dist3D, dst);
        BestQuery q{};
        q.u = u;
        q.v = v;
        q.r = th * dst->scale_factors[pred];
        q.pred = pred;
        qs.push_back(q);
        qd.insert(qd.end(), mps->desc + (size_t)mp * 32, mps->desc + (size_t)mp * 32 + 32);
        slot.push_back(i);
    }
    std::vector<int32_t> out(qs.size());
    const int rc = run_best(m, dst, qs, qd, 0, TH_HIGH, out.data());
    if (rc != ORBX_OK) return rc;
    for (size_t j = 0; j < slot.size(); j++) vnMatch[(size_t)slot[j]] = out[j];
    return ORBX_OK;
}

}  // namespace

// ORBmatcher::SearchBySim3, ORBmatcher.cc:1361-1602
int orbx_search_by_sim3(orbx_matcher* m, const orbx_frame_view* kf1, const int32_t* mp1, const uint8_t* already1,
                        const orbx_frame_view* kf2, const int32_t* mp2, const uint8_t* already2,
                        const orbx_mappoints* mps, float s12, const float* R12, const float* t12, float th,
                        int32_t* matches12, int* nfound) {
    const CallClock clock_(m);
    if (!m || !kf1 || !kf2 || !mp1 || !mp2 || !R12 || !t12 || !matches12 || !nfound || !mps_ok(mps, false))
        return fail(ORBX_ERR_ARG, "null argument");
    if (kf1->nlevels < 2 || kf2->nlevels < 2) return fail(ORBX_ERR_ARG, "need >= 2 pyramid levels");
    // sR12 = s12*R12; sR21 = (1.0/s12)*R12^T (a float Mat scaled by (float)(1/s12)); t21 = -sR21*t12
    float sR12[9], sR21[9], t21[3];
    const float inv = (float)(1.0 / s12);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            sR12[3 * r + c] = s12 * R12[3 * r + c];
            sR21[3 * r + c] = R12[3 * c + r] * inv;
        }
    for (int r = 0; r < 3; r++) t21[r] = -(sR21[3 * r] * t12[0] + sR21[3 * r + 1] * t12[1] + sR21[3 * r + 2] * t12[2]);
    std::vector<int32_t> vnMatch1, vnMatch2;
    int rc = sim3_direction(m, kf1, mp1, already1, kf2, mps, sR21, t21, th, vnMatch1);
    if (rc != ORBX_OK) return rc;
    rc = sim3_direction(m, kf2, mp2, already2, kf1, mps, sR12, t12, th, vnMatch2);
    if (rc != ORBX_OK) return rc;
    int n = 0;
    for (int i1 = 0; i1 < kf1->n; i1++) {  // mutual check (cc:1547-1560)
        const int idx2 = vnMatch1[(size_t)i1];
        if (idx2 >= 0 && vnMatch2[(size_t)idx2] == i1) {
            matches12[i1] = mp2[idx2];
            n++;
        }
    }
    *nfound = n;
    return ORBX_OK;
}

// MapPoint::ComputeDistinctiveDescriptors, MapPoint.cc:295-360, batched over MapPoints
int orbx_compute_distinctive_descriptors_device(int nmp, const int32_t* d_off, const uint8_t* d_desc, int32_t* d_best,
                                                uint8_t* d_out_desc, void* stream) {
    if (nmp < 0 || (nmp && (!d_off || !d_desc || !d_best))) return fail(ORBX_ERR_ARG, "null argument");
    HIP_TRY(launch_distinctive(nmp, d_off, d_desc, d_best, d_out_desc, (hipStream_t)stream));
    return ORBX_OK;
}

int orbx_compute_distinctive_descriptors(int device, int nmp, const int32_t* off, const uint8_t* desc, int32_t* best,
                                         uint8_t* out_desc) {
    if (nmp < 0 || (nmp && (!off || !best))) return fail(ORBX_ERR_ARG, "null argument");
    if (nmp == 0) return ORBX_OK;
    const int total = off[nmp];
    if (total < 0 || (total && !desc)) return fail(ORBX_ERR_ARG, "bad observation offsets");
    for (int k = 0; k < nmp; k++)
        if (off[k + 1] < off[k] || off[k] < 0) return fail(ORBX_ERR_ARG, "bad observation offsets");
    HIP_TRY(hipSetDevice(device));
    char* d = nullptr;
    const size_t bo = pad(sizeof(int32_t) * (nmp + 1)), bd = pad((size_t)total * 32), bb = pad(sizeof(int32_t) * nmp),
                 bx = pad((size_t)nmp * 32);
    HIP_TRY(hipMalloc((void**)&d, bo + bd + bb + bx));
    int32_t* d_off = (int32_t*)d;
    uint8_t* d_desc = (uint8_t*)(d + bo);
    int32_t* d_best = (int32_t*)(d + bo + bd);
    uint8_t* d_out = (uint8_t*)(d + bo + bd + bb);
    hipError_t e = hipMemcpy(d_off, off, sizeof(int32_t) * (nmp + 1), hipMemcpyHostToDevice);
    if (e == hipSuccess && total) e = hipMemcpy(d_desc, desc, (size_t)total * 32, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_distinctive(nmp, d_off, d_desc, d_best, d_out, nullptr);
    if (e == hipSuccess) e = hipMemcpy(best, d_best, sizeof(int32_t) * nmp, hipMemcpyDeviceToHost);
    if (e == hipSuccess && out_desc) e = hipMemcpy(out_desc, d_out, (size_t)nmp * 32, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    HIP_TRY(e);
    return ORBX_OK;
}

// Frame::ComputeStereoMatches, Frame.cc:673-885.  Both entry points fill a StereoBatch
// and run k_stereo_index / k_stereo / k_stereo_outlier (orbx_match.hip).
namespace {

// Level geometry of a stereo pair's pyramids; the two extractors must share it.
int stereo_levels(orbx_extractor* ex_l, orbx_extractor* ex_r, StereoBatch& sb, PyrView& vl, PyrView& vr) {
    int rc = extractor_pyramid(ex_l, &vl, true);
    if (rc != ORBX_OK) return rc;
    rc = extractor_pyramid(ex_r, &vr, true);
    if (rc != ORBX_OK) return rc;
    if (vl.W != vr.W || vl.H != vr.H || vl.L != vr.L || vl.device != vr.device)
        return fail(ORBX_ERR_ARG, "left and right extractors hold pyramids of different geometry");
    for (int l = 0; l < vl.L; l++)
        if (vl.scale[l] != vr.scale[l] || vl.off[l] != vr.off[l] || vl.pitch[l] != vr.pitch[l])
            return fail(ORBX_ERR_ARG, "left and right extractors differ in their scale pyramid");
    sb.rows = vl.h[0];  // mpORBextractorLeft->mvImagePyramid[0].rows (cc:682)
    for (int l = 0; l < vl.L; l++) {
        sb.level_off[l] = vl.off[l];
        sb.level_pitch[l] = vl.pitch[l];
        sb.level_w[l] = vl.w[l];  // mpORBextractorRight->mvImagePyramid[l].cols (cc:810)
        sb.scale[l] = vl.scale[l];
        sb.inv_scale[l] = vl.inv_scale[l];
    }
    sb.fb_l = vl.frame_bytes;
    sb.fb_r = vr.frame_bytes;
    sb.nlevels = vl.L;
    sb.band_cap = sb.cap;  // the (octave, row) index holds every right keypoint once
    return ORBX_OK;
}

// Level 0 of extractions that read it in place: the caller's frames (k_stereo's SAD
// window at octave 0 reads them there).
void stereo_level0(StereoBatch& sb, const PyrView& vl, const PyrView& vr, int left_frame, int right_frame) {
    sb.l0_l = vl.l0 ? vl.l0 + (size_t)left_frame * vl.l0_fp : nullptr;
    sb.l0_r = vr.l0 ? vr.l0 + (size_t)right_frame * vr.l0_fp : nullptr;
    sb.l0_fp_l = vl.l0_fp;
    sb.l0_fp_r = vr.l0_fp;
    sb.l0_pitch_l = vl.l0_pitch;
    sb.l0_pitch_r = vr.l0_pitch;
}

// words of the per-pair (octave, row) offsets + row coverage counts (StereoBatch::row_off)
size_t stereo_off_words(const StereoBatch& sb) { return (size_t)sb.nlevels * sb.rows + 1 + sb.rows; }

size_t stereo_scratch(const StereoBatch& sb, int batch) {
    return pad(sizeof(int32_t) * (size_t)batch * stereo_off_words(sb)) +
           pad(sizeof(int32_t) * (size_t)batch * sb.band_cap) + pad(sizeof(StereoResult) * (size_t)batch * sb.cap);
}

}  // namespace

int orbx_compute_stereo_matches(orbx_matcher* m, orbx_extractor* ex_left, int left_frame, orbx_extractor* ex_right,
                                int right_frame, const orbx_frame_view* left, const orbx_keypoint* keys_r,
                                const uint8_t* desc_r, int n_right, float max_disparity, float* u_right,
                                float* depth) {
    const CallClock clock_(m);
    if (!m || !ex_left || !ex_right || !left || !u_right || !depth || (n_right && (!keys_r || !desc_r)) ||
        n_right < 0 || left->n < 0)
        return fail(ORBX_ERR_ARG, "null argument");
    const int N = left->n;
    for (int i = 0; i < N; i++) {
        u_right[i] = -1.0f;
        depth[i] = -1.0f;
    }
    if (N == 0) return ORBX_OK;
    StereoBatch sb{};
    sb.cap = std::max(N, n_right);
    if (sb.cap > 8192) return fail(ORBX_ERR_UNSUPPORTED, "more than 8192 keypoints per image");
    PyrView vl, vr;
    int rc = stereo_levels(ex_left, ex_right, sb, vl, vr);
    if (rc != ORBX_OK) return rc;
    if (left_frame < 0 || left_frame >= vl.nframes || right_frame < 0 || right_frame >= vr.nframes)
        return fail(ORBX_ERR_ARG, "frame index outside the extractor's last batch");
    for (int i = 0; i < N; i++)
        if (left->keys[i].y < 0 || (int)left->keys[i].y >= sb.rows || left->keys[i].octave < 0 ||
            left->keys[i].octave >= vl.L)
            return fail(ORBX_ERR_ARG, "left keypoint outside the pyramid");
    for (int i = 0; i < n_right; i++)
        if (keys_r[i].octave < 0 || keys_r[i].octave >= vl.L) return fail(ORBX_ERR_ARG, "right keypoint octave");
    sb.pyr_l = vl.base + (size_t)left_frame * vl.frame_bytes;
    sb.pyr_r = vr.base + (size_t)right_frame * vr.frame_bytes;
    stereo_level0(sb, vl, vr, left_frame, right_frame);
    sb.bf = left->bf;
    sb.max_d = max_disparity;
    HIP_TRY(hipSetDevice(m->device));
    const size_t need = pad(sizeof(orbx_keypoint) * sb.cap) * 2 + pad((size_t)sb.cap * 32) * 2 + 2 * pad(sizeof(int32_t)) +
                        2 * pad(sizeof(float) * sb.cap) + stereo_scratch(sb, 1);
    HIP_TRY(m->arena.reserve(need));
    m->arena.used = 0;
    auto* d_kl = m->arena.take<orbx_keypoint>(sb.cap);
    auto* d_dl = m->arena.take<uint8_t>((size_t)sb.cap * 32);
    auto* d_kr = m->arena.take<orbx_keypoint>(sb.cap);
    auto* d_dr = m->arena.take<uint8_t>((size_t)sb.cap * 32);
    auto* d_nl = m->arena.take<int32_t>(1);
    auto* d_nr = m->arena.take<int32_t>(1);
    auto* d_ur = m->arena.take<float>(sb.cap);
    auto* d_dp = m->arena.take<float>(sb.cap);
    sb.row_off = m->arena.take<int32_t>(stereo_off_words(sb));
    sb.row_idx = m->arena.take<int32_t>((size_t)sb.band_cap);
    sb.res = m->arena.take<StereoResult>(sb.cap);
    // the extractors' streams produced the pyramids: order this stream after them
    HIP_TRY(hipStreamSynchronize(vl.stream));
    if (vr.stream != vl.stream) HIP_TRY(hipStreamSynchronize(vr.stream));
    hipStream_t s = m->stream;
    m->arena.up(d_kl, left->keys, sizeof(orbx_keypoint) * N);
    m->arena.up(d_dl, left->desc, (size_t)N * 32);
    if (n_right) {
        m->arena.up(d_kr, keys_r, sizeof(orbx_keypoint) * n_right);
        m->arena.up(d_dr, desc_r, (size_t)n_right * 32);
    }
    const int32_t nl = N, nr = n_right;
    m->arena.up(d_nl, &nl, sizeof(nl));
    m->arena.up(d_nr, &nr, sizeof(nr));
    sb.keys_l = d_kl;
    sb.desc_l = d_dl;
    sb.n_l = d_nl;
    sb.keys_r = d_kr;
    sb.desc_r = d_dr;
    sb.n_r = d_nr;
    sb.u_right = d_ur;
    sb.depth = d_dp;
    HIP_TRY(m->arena.flush(s));
    HIP_TRY(launch_stereo(sb, 1, s));
    HIP_TRY(m->arena.down(u_right, d_ur, sizeof(float) * N, s));
    HIP_TRY(m->arena.down(depth, d_dp, sizeof(float) * N, s));
    HIP_TRY(m->arena.sync(s));
    return ORBX_OK;
}

int orbx_compute_stereo_matches_batch_device(orbx_matcher* m, orbx_extractor* ex_left, int left_frame0,
                                             orbx_extractor* ex_right, int right_frame0, int batch,
                                             const orbx_keypoint* d_kps_l, const uint8_t* d_desc_l,
                                             const int32_t* d_n_l, const orbx_keypoint* d_kps_r,
                                             const uint8_t* d_desc_r, const int32_t* d_n_r, int cap, float bf,
                                             float max_disparity, float* d_u_right, float* d_depth, void* stream) {
    if (!m || !ex_left || !ex_right || batch < 0 || cap <= 0) return fail(ORBX_ERR_ARG, "bad argument");
    if (batch == 0) return ORBX_OK;
    if (!d_kps_l || !d_desc_l || !d_n_l || !d_kps_r || !d_desc_r || !d_n_r || !d_u_right || !d_depth)
        return fail(ORBX_ERR_ARG, "null buffer");
    if (cap > 8192) return fail(ORBX_ERR_UNSUPPORTED, "cap above 8192 keypoints per image");
    StereoBatch sb{};
    sb.cap = cap;
    PyrView vl, vr;
    int rc = stereo_levels(ex_left, ex_right, sb, vl, vr);
    if (rc != ORBX_OK) return rc;
    if (left_frame0 < 0 || left_frame0 + batch > vl.nframes || right_frame0 < 0 || right_frame0 + batch > vr.nframes)
        return fail(ORBX_ERR_ARG, "pair range outside the extractors' last batches");
    HIP_TRY(hipSetDevice(m->device));
    hipStream_t s = stream ? (hipStream_t)stream : m->stream;
    const size_t need = stereo_scratch(sb, batch);
    if (m->dscr_cap < need) {
        HIP_TRY(hipStreamSynchronize(s));
        if (m->dscr) HIP_TRY(hipFree(m->dscr));
        m->dscr = nullptr;
        m->dscr_cap = 0;
        HIP_TRY(hipMalloc((void**)&m->dscr, need));
        m->dscr_cap = need;
    }
    char* p = m->dscr;
    sb.row_off = (int32_t*)p;
    p += pad(sizeof(int32_t) * (size_t)batch * stereo_off_words(sb));
    sb.row_idx = (int32_t*)p;
    p += pad(sizeof(int32_t) * (size_t)batch * sb.band_cap);
    sb.res = (StereoResult*)p;
    sb.keys_l = d_kps_l;
    sb.desc_l = d_desc_l;
    sb.n_l = d_n_l;
    sb.keys_r = d_kps_r;
    sb.desc_r = d_desc_r;
    sb.n_r = d_n_r;
    sb.pyr_l = vl.base + (size_t)left_frame0 * vl.frame_bytes;
    sb.pyr_r = vr.base + (size_t)right_frame0 * vr.frame_bytes;
    stereo_level0(sb, vl, vr, left_frame0, right_frame0);
    sb.bf = bf;
    sb.max_d = max_disparity;
    sb.u_right = d_u_right;
    sb.depth = d_depth;
    hipEvent_t* ev = m->ev[m->ncalls % orbx_matcher::kRing];
    if (m->timing) {
        for (int i = 0; i < 2; i++)
            if (!ev[i]) HIP_TRY(hipEventCreate(&ev[i]));
        HIP_TRY(hipEventRecord(ev[0], s));
    }
    HIP_TRY(launch_stereo(sb, batch, s));
    if (m->timing) {
        HIP_TRY(hipEventRecord(ev[1], s));
        m->ncalls++;
    }
    return ORBX_OK;
}

}  // extern "C"
