// orbx_api.cpp -- the extern "C" boundary (include/orbx.h) over the HIP kernels.
//
// One orbx_extractor == one reference ORBextractor instance: it owns a HIP stream,
// the device plan for the last frame size, device buffers sized for the largest
// batch seen, and (like the reference's mvImagePyramid) keeps the pyramid of the
// last extraction until the next call.  No function throws across the ABI.
#include <atomic>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "orbx.h"
#include "orbx_error.h"
#include "orbx_kernels.h"

using namespace orbx;

namespace {

int fail(int code, const char* what) {
    set_last_error(what ? what : "");
    return code;
}

int hip_fail(hipError_t e, const char* where) {
    set_last_error(std::string(where) + ": " + hipGetErrorString(e));
    return ORBX_ERR_HIP;
}

#define HIP_TRY(expr)                                      \
    do {                                                   \
        hipError_t _e = (expr);                            \
        if (_e != hipSuccess) return hip_fail(_e, #expr);  \
    } while (0)

template <typename T>
hipError_t dalloc(T** p, size_t n) {
    if (n == 0) n = 1;
    return hipMalloc((void**)p, sizeof(T) * n);
}

}  // namespace

struct orbx_extractor {
    int device = 0;
    OrbParams prm{};
    hipStream_t stream = nullptr;
    Plan plan;
    DeviceBuffers db;
    // Stage timing: a ring of event sets, one per timed call, so a whole timed loop is
    // measured without synchronising inside it; stage_times averages the ring.
    static constexpr int kRing = 64;
    // orbx_extractor_set_level0_in_place: level 0 stays in the caller's device frames (no
    // copy into the pyramid) when they are aligned for it; l0_* describe the last call's
    bool l0_in_place = false;
    const uint8_t* l0 = nullptr;
    size_t l0_fp = 0, l0_pitch = 0;
    bool timing = false;
    int timing_stage = -1;  // -1: every stage boundary; s >= 0: only stage s's two events
    hipEvent_t ev[kRing][kStages + 1] = {};
    long long ncalls = 0;
    // host-API staging
    uint8_t* d_in = nullptr;
    size_t d_in_bytes = 0;
    // pinned mirrors of d_in / d_kps / d_desc / d_n: host frames are packed here and
    // uploaded in one copy (a 2-D copy of an odd-width frame goes row by row), results
    // come back through them
    uint8_t* h_in = nullptr;
    orbx_keypoint* h_kps = nullptr;
    uint8_t* h_desc = nullptr;
    int* h_n = nullptr;
    int* h_status = nullptr;
    // the same pinned buffers as the device sees them (host-mapped, coherent): the single
    // host calls read their frames and write their results through these, no DMA copies
    const uint8_t* h_in_dev = nullptr;
    orbx_keypoint* h_kps_dev = nullptr;
    uint8_t* h_desc_dev = nullptr;
    int* h_n_dev = nullptr;
    int* h_status_dev = nullptr;
    orbx_keypoint* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int* d_n = nullptr;
    size_t d_out_cap = 0;  // keypoint slots
    int d_n_cap = 0;
    int last_batch = 0;
    bool have_pyramid = false;
    hipStream_t last_stream = nullptr;  // stream of the last extraction (status reads order after it)
    // orbx_extractor_set_stage_event: recorded after stage `stage_after` of every extraction
    hipEvent_t stage_ev = nullptr;
    int stage_after = 0;
    double last_call_us = 0.0;  // wall time of the newest host-API extraction (orbx_extractor_last_call_us)
};

namespace {

void free_buffers(DeviceBuffers& db) {
    void* ptrs[] = {db.lv, db.cells, db.rtab, db.pyr, db.blur, db.score, db.slots, db.cell_count,
                    db.keys, db.key_node, db.kept, db.kept_count, db.status, db.oct_stamps, db.dt_list,
                    db.dt_tile};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    db = DeviceBuffers();
}

// (Re)plan for a frame size and make sure buffers hold `batch` frames.
int prepare(orbx_extractor* ex, int W, int H, int batch) {
    HIP_TRY(hipSetDevice(ex->device));
    const bool same_size = ex->plan.ok && ex->plan.W == W && ex->plan.H == H;
    if (!same_size) {
        HIP_TRY(hipStreamSynchronize(ex->stream));
        free_buffers(ex->db);
        ex->have_pyramid = false;
        if (!make_plan(ex->plan, ex->prm, W, H)) return fail(ORBX_ERR_UNSUPPORTED, ex->plan.why);
    }
    if (ex->db.batch_cap >= batch && same_size) return ORBX_OK;
    HIP_TRY(hipStreamSynchronize(ex->stream));
    const Plan& p = ex->plan;
    DeviceBuffers& db = ex->db;
    free_buffers(db);
    ex->have_pyramid = false;
    const size_t B = (size_t)batch;
    HIP_TRY(dalloc(&db.lv, kMaxLevels));
    HIP_TRY(dalloc(&db.cells, p.cells.size()));
    HIP_TRY(dalloc(&db.rtab, p.rtab.size()));
    // slack: k_describe's dword patch loads may reach a few bytes past a level's last row
    HIP_TRY(dalloc(&db.pyr, B * (size_t)p.pyr_frame_bytes + 65536));
    HIP_TRY(dalloc(&db.blur, B * (size_t)p.pyr_frame_bytes + 65536));
    HIP_TRY(dalloc(&db.score, B * (size_t)p.pyr_frame_bytes + 65536));  // k_fast_cells reads past windows
    HIP_TRY(dalloc(&db.slots, B * (size_t)p.slots_per_frame));
    HIP_TRY(dalloc(&db.cell_count, B * p.cells.size()));
    HIP_TRY(dalloc(&db.keys, B * (size_t)p.keys_per_frame));
    HIP_TRY(dalloc(&db.key_node, B * (size_t)p.keys_per_frame));
    HIP_TRY(dalloc(&db.kept, B * (size_t)p.kept_per_frame));
    HIP_TRY(dalloc(&db.kept_count, B * (size_t)p.L));
    HIP_TRY(dalloc(&db.dt_list, B * (size_t)p.kept_per_frame));
    HIP_TRY(dalloc(&db.dt_tile, B * (size_t)p.tiles_total));
    HIP_TRY(dalloc(&db.status, B));
    if (tuning(Tune::OctStamps, 0) > 0) HIP_TRY(dalloc(&db.oct_stamps, B * (size_t)p.L * 16));  // kOctStampWords
    HIP_TRY(hipMemcpyAsync(db.lv, p.lv, sizeof(LevelGeom) * kMaxLevels, hipMemcpyHostToDevice, ex->stream));
    HIP_TRY(hipMemcpyAsync(db.cells, p.cells.data(), sizeof(CellGeom) * p.cells.size(), hipMemcpyHostToDevice,
                           ex->stream));
    HIP_TRY(hipMemcpyAsync(db.rtab, p.rtab.data(), sizeof(int16_t) * p.rtab.size(), hipMemcpyHostToDevice,
                           ex->stream));
    HIP_TRY(hipMemsetAsync(db.pyr, 0, B * (size_t)p.pyr_frame_bytes, ex->stream));
    HIP_TRY(hipMemsetAsync(db.blur, 0, B * (size_t)p.pyr_frame_bytes, ex->stream));
    HIP_TRY(hipStreamSynchronize(ex->stream));
    db.batch_cap = batch;
    return ORBX_OK;
}

int max_kps_of(const Plan& p) {
    int s = 0;
    for (int l = 0; l < p.L; l++) s += p.lv[l].ncap;
    return s;
}

int run_device(orbx_extractor* ex, int batch, const uint8_t* d_imgs, size_t frame_pitch, int W, int H,
               size_t stride, orbx_keypoint* d_kps, uint8_t* d_desc, int cap, int* d_n, hipStream_t stream,
               bool allow_inplace = true, int* status_out = nullptr) {
    int rc = prepare(ex, W, H, batch);
    if (rc != ORBX_OK) return rc;
    hipEvent_t* ev = nullptr;
    hipEvent_t sel[kStages + 1] = {};
    if (ex->timing) {
        hipEvent_t* slot = ex->ev[ex->ncalls % orbx_extractor::kRing];
        for (int i = 0; i <= kStages; i++)
            if (!slot[i]) HIP_TRY(hipEventCreate(&slot[i]));
        ev = slot;
        if (ex->timing_stage >= 0) {  // only the timed stage's boundaries are recorded
            sel[ex->timing_stage] = slot[ex->timing_stage];
            sel[ex->timing_stage + 1] = slot[ex->timing_stage + 1];
            ev = sel;
        }
    }
    const bool inplace = allow_inplace && ex->l0_in_place && !ex->plan.desc_tiles && (uintptr_t)d_imgs % 16 == 0 &&
                         stride % 64 == 0 && frame_pitch % 16 == 0;
    hipError_t e = launch_extract(ex->plan, ex->db, batch, d_imgs, frame_pitch, stride, d_kps, d_desc, cap, d_n,
                                  stream, ev, ex->stage_ev, ex->stage_after, inplace, status_out);
    ex->l0 = inplace ? d_imgs : nullptr;
    ex->l0_fp = frame_pitch;
    ex->l0_pitch = stride;
    if (e != hipSuccess) return hip_fail(e, "launch_extract");
    if (ex->db.oct_stamps) {  // diagnostics: per-level k_octree phase times (us) to stderr
        const int L = ex->plan.L;
        constexpr int W = 16;  // kOctStampWords
        std::vector<unsigned long long> h((size_t)batch * L * W);
        HIP_TRY(hipStreamSynchronize(stream));
        HIP_TRY(hipMemcpy(h.data(), ex->db.oct_stamps, h.size() * 8, hipMemcpyDeviceToHost));
        for (int l = 0; l < L; l++) {
            double ph[4] = {0, 0, 0, 0}, mx = 0, n = 0, g1 = 0, g2 = 0, rk = 0;
            for (int f = 0; f < batch; f++) {
                const unsigned long long* r = &h[((size_t)f * L + l) * W];
                rk += (double)r[8] * 0.01;
                for (int k = 0; k < 4; k++) ph[k] += (double)(r[k + 1] - r[k]) * 0.01;
                const double tot = (double)(r[4] - r[0]) * 0.01;
                mx = tot > mx ? tot : mx;
                n += (double)r[6];
                g1 += (double)r[7];
                g2 += (double)r[5];
            }
            fprintf(stderr,
                    "[orbx oct] L%d keys %.0f | gather %.1f passes %.1f (%.1f it) final %.1f (%.1f it, ranking %.1f) out %.1f"
                    " | max %.1f us\n",
                    l, n / batch, ph[0] / batch, ph[1] / batch, g1 / batch, ph[2] / batch, (g2 - g1) / batch, rk / batch,
                    ph[3] / batch, mx);
        }
    }
    if (ex->timing) ex->ncalls++;
    ex->last_batch = batch;
    ex->have_pyramid = true;
    ex->last_stream = stream;
    return ORBX_OK;
}

// The octree status words of the last `batch` frames: read back from the device, or taken
// from `known` (the host-mapped mirror a host call's describe kernel filled).
int check_status(orbx_extractor* ex, int batch, const int* known = nullptr) {
    std::vector<int> st((size_t)batch);
    if (known)
        std::memcpy(st.data(), known, sizeof(int) * (size_t)batch);
    else
        HIP_TRY(hipMemcpy(st.data(), ex->db.status, sizeof(int) * (size_t)batch, hipMemcpyDeviceToHost));
    for (int b = 0; b < batch; b++)
        if (st[(size_t)b]) {
            char msg[160];
            snprintf(msg, sizeof(msg), "octree kernel reported %s%s (frame %d): keypoints truncated",
                     (st[(size_t)b] & kStatusNodeOverflow) ? "a node-capacity overflow" : "",
                     (st[(size_t)b] & kStatusIterations) ? " an iteration-guard stop" : "", b);
            return fail(ORBX_ERR_STATE, msg);
        }
    return ORBX_OK;
}

// Pinned host memory, mapped into the device's address space and coherent (the GPU does
// not cache it): the host calls' frames are read, and their results written, through the
// device pointer (*dev), so a call needs no DMA copy and one synchronisation.
template <typename T>
hipError_t halloc(T** p, size_t n, T** dev) {
    if (n == 0) n = 1;
    hipError_t e = hipHostMalloc((void**)p, sizeof(T) * n, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return e;
    return hipHostGetDevicePointer((void**)dev, *p, 0);
}

void free_host_staging(orbx_extractor* ex) {
    if (ex->d_in) (void)hipFree(ex->d_in);
    if (ex->d_kps) (void)hipFree(ex->d_kps);
    if (ex->d_desc) (void)hipFree(ex->d_desc);
    if (ex->d_n) (void)hipFree(ex->d_n);
    if (ex->h_in) (void)hipHostFree(ex->h_in);
    if (ex->h_kps) (void)hipHostFree(ex->h_kps);
    if (ex->h_desc) (void)hipHostFree(ex->h_desc);
    if (ex->h_n) (void)hipHostFree(ex->h_n);
    if (ex->h_status) (void)hipHostFree(ex->h_status);
    ex->h_status = nullptr;
    ex->h_in_dev = nullptr;
    ex->h_kps_dev = nullptr;
    ex->h_desc_dev = nullptr;
    ex->h_n_dev = nullptr;
    ex->h_status_dev = nullptr;
    ex->d_in = nullptr;
    ex->d_kps = nullptr;
    ex->d_desc = nullptr;
    ex->d_n = nullptr;
    ex->h_in = nullptr;
    ex->h_kps = nullptr;
    ex->h_desc = nullptr;
    ex->h_n = nullptr;
    ex->d_in_bytes = 0;
    ex->d_out_cap = 0;
    ex->d_n_cap = 0;
}

int ensure_host_staging(orbx_extractor* ex, size_t in_bytes, size_t out_slots, int nframes) {
    if (ex->d_in_bytes < in_bytes) {
        if (ex->d_in) (void)hipFree(ex->d_in);
        if (ex->h_in) (void)hipHostFree(ex->h_in);
        ex->d_in = nullptr;
        ex->h_in = nullptr;
        ex->d_in_bytes = 0;
        HIP_TRY(dalloc(&ex->d_in, in_bytes));
        uint8_t* dev = nullptr;
        HIP_TRY(halloc(&ex->h_in, in_bytes, &dev));
        ex->h_in_dev = dev;
        ex->d_in_bytes = in_bytes;
    }
    if (ex->d_out_cap < out_slots) {
        if (ex->d_kps) (void)hipFree(ex->d_kps);
        if (ex->d_desc) (void)hipFree(ex->d_desc);
        if (ex->h_kps) (void)hipHostFree(ex->h_kps);
        if (ex->h_desc) (void)hipHostFree(ex->h_desc);
        ex->d_kps = nullptr;
        ex->d_desc = nullptr;
        ex->h_kps = nullptr;
        ex->h_desc = nullptr;
        ex->d_out_cap = 0;
        HIP_TRY(dalloc(&ex->d_kps, out_slots));
        HIP_TRY(dalloc(&ex->d_desc, out_slots * 32));
        HIP_TRY(halloc(&ex->h_kps, out_slots, &ex->h_kps_dev));
        HIP_TRY(halloc(&ex->h_desc, out_slots * 32, &ex->h_desc_dev));
        ex->d_out_cap = out_slots;
    }
    if (ex->d_n_cap < nframes) {
        if (ex->d_n) (void)hipFree(ex->d_n);
        if (ex->h_n) (void)hipHostFree(ex->h_n);
        if (ex->h_status) (void)hipHostFree(ex->h_status);
        ex->d_n = nullptr;
        ex->h_n = nullptr;
        ex->h_status = nullptr;
        ex->d_n_cap = 0;
        HIP_TRY(dalloc(&ex->d_n, (size_t)nframes));
        HIP_TRY(halloc(&ex->h_n, (size_t)nframes, &ex->h_n_dev));
        HIP_TRY(halloc(&ex->h_status, (size_t)nframes, &ex->h_status_dev));
        ex->d_n_cap = nframes;
    }
    return ORBX_OK;
}

}  // namespace

int orbx::extractor_pyramid(orbx_extractor* ex, PyrView* v, bool allow_l0) {
    if (!ex || !v) return fail(ORBX_ERR_ARG, "null argument");
    if (!ex->have_pyramid) return fail(ORBX_ERR_STATE, "no extraction yet");
    if (ex->l0 && !allow_l0)
        return fail(ORBX_ERR_STATE, "pyramid level 0 was read in place (orbx_extractor_set_level0_in_place)");
    v->l0 = ex->l0;
    v->l0_fp = (long long)ex->l0_fp;
    v->l0_pitch = (int)ex->l0_pitch;
    const Plan& p = ex->plan;
    v->base = ex->db.pyr;
    v->frame_bytes = p.pyr_frame_bytes;
    v->nframes = ex->last_batch;
    v->W = p.W;
    v->H = p.H;
    v->L = p.L;
    for (int l = 0; l < p.L; l++) {
        v->off[l] = p.lv[l].off;
        v->pitch[l] = p.lv[l].pitch;
        v->w[l] = p.lv[l].w;
        v->h[l] = p.lv[l].h;
        v->scale[l] = ex->prm.scale[l];
        v->inv_scale[l] = ex->prm.inv_scale[l];
    }
    v->device = ex->device;
    v->stream = ex->last_stream;
    return ORBX_OK;
}

extern "C" {

const char* orbx_version(void) { return "orbx 0.1 (gfx950)"; }


int orbx_device_count(int* n) {
    if (!n) return fail(ORBX_ERR_ARG, "null");
    int c = 0;
    HIP_TRY(hipGetDeviceCount(&c));
    *n = c;
    return ORBX_OK;
}

int orbx_extractor_create(const orbx_extractor_params* params, int device, orbx_extractor** out) {
    if (!params || !out) return fail(ORBX_ERR_ARG, "null argument");
    *out = nullptr;
    orbx_extractor* ex = new (std::nothrow) orbx_extractor();
    if (!ex) return fail(ORBX_ERR_ARG, "out of host memory");
    if (!init_params(ex->prm, params->nfeatures, params->scale_factor, params->nlevels, params->ini_th_fast,
                     params->min_th_fast)) {
        delete ex;
        return fail(ORBX_ERR_ARG, "invalid ORB parameters");
    }
    ex->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ex->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = upload_constants(ex->prm);
    if (e != hipSuccess) {
        delete ex;
        return hip_fail(e, "orbx_extractor_create");
    }
    *out = ex;
    return ORBX_OK;
}

void orbx_extractor_destroy(orbx_extractor* ex) {
    if (!ex || orbx::unloading()) return;
    (void)hipSetDevice(ex->device);
    if (ex->stream) (void)hipStreamSynchronize(ex->stream);
    free_buffers(ex->db);
    free_host_staging(ex);
    for (auto& slot : ex->ev)
        for (auto& e : slot)
            if (e) (void)hipEventDestroy(e);
    if (ex->stage_ev) (void)hipEventDestroy(ex->stage_ev);
    if (ex->stream) (void)hipStreamDestroy(ex->stream);
    delete ex;
}

int orbx_extractor_levels(const orbx_extractor* ex, int* nlevels, float* scale, float* inv_scale, float* sigma2,
                          float* inv_sigma2) {
    if (!ex) return fail(ORBX_ERR_ARG, "null extractor");
    const int L = ex->prm.nlevels;
    if (nlevels) *nlevels = L;
    if (scale) std::memcpy(scale, ex->prm.scale, sizeof(float) * L);
    if (inv_scale) std::memcpy(inv_scale, ex->prm.inv_scale, sizeof(float) * L);
    if (sigma2) std::memcpy(sigma2, ex->prm.sigma2, sizeof(float) * L);
    if (inv_sigma2) std::memcpy(inv_sigma2, ex->prm.inv_sigma2, sizeof(float) * L);
    return ORBX_OK;
}

int orbx_extractor_features_per_level(const orbx_extractor* ex, int* features) {
    if (!ex || !features) return fail(ORBX_ERR_ARG, "null argument");
    std::memcpy(features, ex->prm.features, sizeof(int) * ex->prm.nlevels);
    return ORBX_OK;
}

int orbx_extractor_max_keypoints(orbx_extractor* ex, int width, int height, int* max_kps) {
    if (!ex || !max_kps) return fail(ORBX_ERR_ARG, "null argument");
    Plan p;
    if (!make_plan(p, ex->prm, width, height)) return fail(ORBX_ERR_UNSUPPORTED, p.why);
    *max_kps = max_kps_of(p);
    return ORBX_OK;
}

void* orbx_extractor_stream(orbx_extractor* ex) { return ex ? (void*)ex->stream : nullptr; }

int orbx_extractor_set_stage_event(orbx_extractor* ex, int stage, void** event) {
    if (!ex || stage < 0 || stage > 4) return fail(ORBX_ERR_ARG, "stage is 0 (off) or 1..4");
    HIP_TRY(hipSetDevice(ex->device));
    if (!ex->stage_ev) HIP_TRY(hipEventCreateWithFlags(&ex->stage_ev, hipEventDisableTiming));
    ex->stage_after = stage;
    if (event) *event = stage > 0 ? (void*)ex->stage_ev : nullptr;
    return ORBX_OK;
}

int orbx_stream_wait_event(void* stream, void* event) {
    if (!event) return fail(ORBX_ERR_ARG, "null event");
    HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
    return ORBX_OK;
}

int orbx_stream_create(int device, int cu_stride, int priority, void** stream) {
    if (!stream || cu_stride < 1) return fail(ORBX_ERR_ARG, "bad argument");
    if (cu_stride > 1 && priority != 0) return fail(ORBX_ERR_ARG, "a CU-masked stream has the default priority");
    *stream = nullptr;
    HIP_TRY(hipSetDevice(device));
    int ncu = 0;
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
    hipStream_t s = nullptr;
    if (cu_stride == 1) {
        HIP_TRY(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
    } else {
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; i += cu_stride) mask[(size_t)i / 32] |= 1u << (i % 32);
        HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    }
    *stream = (void*)s;
    return ORBX_OK;
}

int orbx_stream_destroy(void* stream) {
    if (!stream) return fail(ORBX_ERR_ARG, "null stream");
    if (orbx::unloading()) return ORBX_OK;
    HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return ORBX_OK;
}

int orbx_extractor_status(orbx_extractor* ex, int batch, int* flags, int* any) {
    if (!ex || batch < 0) return fail(ORBX_ERR_ARG, "bad argument");
    if (!ex->have_pyramid) return fail(ORBX_ERR_STATE, "no extraction yet");
    if (batch > ex->last_batch) return fail(ORBX_ERR_ARG, "batch exceeds the last extraction");
    HIP_TRY(hipSetDevice(ex->device));
    HIP_TRY(hipStreamSynchronize(ex->last_stream));
    std::vector<int> st((size_t)(batch > 0 ? batch : 1));
    if (batch > 0)
        HIP_TRY(hipMemcpy(st.data(), ex->db.status, sizeof(int) * (size_t)batch, hipMemcpyDeviceToHost));
    int a = 0;
    for (int b = 0; b < batch; b++) a |= st[(size_t)b];
    if (flags) std::memcpy(flags, st.data(), sizeof(int) * (size_t)batch);
    if (any) *any = a;
    return ORBX_OK;
}

int orbx_extractor_status_device(orbx_extractor* ex, const int32_t** d_status) {
    if (!ex || !d_status) return fail(ORBX_ERR_ARG, "null argument");
    if (!ex->have_pyramid) return fail(ORBX_ERR_STATE, "no extraction yet");
    *d_status = ex->db.status;
    return ORBX_OK;
}

int orbx_extractor_set_level0_in_place(orbx_extractor* ex, int enable) {
    if (!ex) return fail(ORBX_ERR_ARG, "null extractor");
    ex->l0_in_place = enable != 0;
    return ORBX_OK;
}

int orbx_extractor_set_node_capacity(orbx_extractor* ex, int cap) {
    if (!ex || cap < 0) return fail(ORBX_ERR_ARG, "bad argument");
    HIP_TRY(hipSetDevice(ex->device));
    // the buffers freed below include the pyramids, which consumers on other streams read
    // (orbx_compute_stereo_matches_batch_device on a matcher's stream): a test hook, so
    // the whole device is drained rather than only this extractor's streams
    HIP_TRY(hipDeviceSynchronize());
    ex->prm.node_cap_limit = cap;
    free_buffers(ex->db);  // replanned (and reallocated) by the next extraction
    ex->plan = Plan();
    ex->have_pyramid = false;
    return ORBX_OK;
}

int orbx_extractor_set_timing(orbx_extractor* ex, int enable) {
    if (!ex) return fail(ORBX_ERR_ARG, "null extractor");
    if (enable < 0 || enable > 1 + kStages - 1) return fail(ORBX_ERR_ARG, "timing: 0, 1 or 2 + stage (0..4)");
    ex->timing = enable != 0;
    ex->timing_stage = enable >= 2 ? enable - 2 : -1;
    ex->ncalls = 0;
    return ORBX_OK;
}

int orbx_extractor_stage_times(orbx_extractor* ex, int max_stages, const char** names, float* ms, int* n_stages) {
    if (!ex) return fail(ORBX_ERR_ARG, "null extractor");
    if (ex->ncalls == 0) return fail(ORBX_ERR_STATE, "no timed extraction yet");
    const long long last = ex->ncalls - 1;
    const int nslots = ex->ncalls < orbx_extractor::kRing ? (int)ex->ncalls : orbx_extractor::kRing;
    if (ex->timing_stage >= 0) {  // one stage timed
        const int st = ex->timing_stage;
        HIP_TRY(hipEventSynchronize(ex->ev[last % orbx_extractor::kRing][st + 1]));
        double sum = 0.0;
        for (int k = 0; k < nslots; k++) {
            hipEvent_t* e = ex->ev[(last - k) % orbx_extractor::kRing];
            float t = 0.f;
            HIP_TRY(hipEventElapsedTime(&t, e[st], e[st + 1]));
            sum += t;
        }
        if (max_stages >= 1) {
            if (names) names[0] = kStageNames[st];
            if (ms) ms[0] = (float)(sum / nslots);
        }
        if (n_stages) *n_stages = max_stages >= 1 ? 1 : 0;
        return ORBX_OK;
    }
    HIP_TRY(hipEventSynchronize(ex->ev[last % orbx_extractor::kRing][kStages - 1]));
    int n = kStages < max_stages ? kStages : max_stages;
    for (int i = 0; i < n; i++) {
        double sum = 0.0;
        for (int k = 0; k < nslots; k++) {
            hipEvent_t* e = ex->ev[(last - k) % orbx_extractor::kRing];
            float t = 0.f;
            if (i < kStages - 1)
                HIP_TRY(hipEventElapsedTime(&t, e[i], e[i + 1]));
            else
                HIP_TRY(hipEventElapsedTime(&t, e[0], e[kStages - 1]));
            sum += t;
        }
        if (names) names[i] = kStageNames[i];
        if (ms) ms[i] = (float)(sum / nslots);
    }
    if (n_stages) *n_stages = n;
    return ORBX_OK;
}

int orbx_extract_batch_device(orbx_extractor* ex, int batch, const uint8_t* d_imgs, size_t frame_pitch, int width,
                              int height, size_t stride, orbx_keypoint* d_kps, uint8_t* d_desc, int cap,
                              int* d_n_per_frame, void* stream) {
    if (!ex || batch < 0 || cap < 0) return fail(ORBX_ERR_ARG, "bad argument");
    if (batch == 0) return ORBX_OK;
    if (width <= 0 || height <= 0 || !d_imgs) return ORBX_EMPTY;  // ORBextractor.cc:1517-1518
    if (stride < (size_t)width || !d_kps || !d_desc || !d_n_per_frame) return fail(ORBX_ERR_ARG, "bad buffers");
    hipStream_t s = stream ? (hipStream_t)stream : ex->stream;
    return run_device(ex, batch, d_imgs, frame_pitch, width, height, stride, d_kps, d_desc, cap, d_n_per_frame, s);
}

namespace {
// Scoped: the enclosing host call's wall time into ex->last_call_us.
struct CallClock {
    orbx_extractor* ex;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    ~CallClock() {
        if (ex) ex->last_call_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    }
};
}  // namespace

double orbx_extractor_last_call_us(const orbx_extractor* ex) { return ex ? ex->last_call_us : -1.0; }

int orbx_extract_batch(orbx_extractor* ex, int batch, const uint8_t* const* imgs, int width, int height,
                       size_t stride, orbx_keypoint* kps, uint8_t* desc, int cap, int* n_per_frame) {
    CallClock clock{ex};
    if (!ex || batch < 0 || cap < 0 || !imgs) return fail(ORBX_ERR_ARG, "bad argument");
    if (batch == 0) return ORBX_OK;
    if (width <= 0 || height <= 0) return ORBX_EMPTY;
    if (stride < (size_t)width || !n_per_frame) return fail(ORBX_ERR_ARG, "bad buffers");
    HIP_TRY(hipSetDevice(ex->device));
    const size_t fbytes = (size_t)width * height;
    int rc = ensure_host_staging(ex, fbytes * batch, (size_t)batch * (cap > 0 ? cap : 1), batch);
    if (rc != ORBX_OK) return rc;
    // the previous call's downloads into the pinned mirrors completed at its final sync
    for (int b = 0; b < batch; b++) {
        uint8_t* dst = ex->h_in + fbytes * b;
        if (stride == (size_t)width) {
            std::memcpy(dst, imgs[b], fbytes);
        } else {
            for (int y = 0; y < height; y++) std::memcpy(dst + (size_t)y * width, imgs[b] + (size_t)y * stride, width);
        }
    }
    // Default: the pyramid kernel reads the frames from the mapped pinned buffer and the
    // describe kernel writes keypoints, descriptors, counts and status words straight into
    // mapped pinned memory -- no DMA copy in either direction and one synchronisation per
    // call.  Switch extract_dma = 1 (orbx_debug_set): the round-4 path (upload copy, results
    // read back by copies; tests/test_gpu_extract.py runs both).
    const bool dma = tuning(Tune::ExtractDma, 0) > 0;
    if (!dma) {
        rc = run_device(ex, batch, ex->h_in_dev, fbytes, width, height, (size_t)width, ex->h_kps_dev, ex->h_desc_dev,
                        cap > 0 ? cap : 1, ex->h_n_dev, ex->stream, false, ex->h_status_dev);
        if (rc != ORBX_OK) return rc;
        HIP_TRY(hipStreamSynchronize(ex->stream));
        std::memcpy(n_per_frame, ex->h_n, sizeof(int) * batch);
        rc = check_status(ex, batch, ex->h_status);
        if (rc != ORBX_OK) return rc;
        int overflow = 0;
        for (int b = 0; b < batch; b++) {
            const int n = n_per_frame[b] < cap ? n_per_frame[b] : cap;
            if (n_per_frame[b] > cap) overflow = 1;
            if (n <= 0) continue;
            if (kps) std::memcpy(kps + (size_t)b * cap, ex->h_kps + (size_t)b * cap, sizeof(orbx_keypoint) * n);
            if (desc) std::memcpy(desc + (size_t)b * cap * 32, ex->h_desc + (size_t)b * cap * 32, (size_t)n * 32);
        }
        return overflow ? fail(ORBX_ERR_CAPACITY, "more keypoints than cap") : ORBX_OK;
    }
    HIP_TRY(hipMemcpyAsync(ex->d_in, ex->h_in, fbytes * batch, hipMemcpyHostToDevice, ex->stream));
    rc = run_device(ex, batch, ex->d_in, fbytes, width, height, (size_t)width, ex->d_kps, ex->d_desc,
                    cap > 0 ? cap : 1, ex->d_n, ex->stream);
    if (rc != ORBX_OK) return rc;
    HIP_TRY(hipMemcpyAsync(ex->h_n, ex->d_n, sizeof(int) * batch, hipMemcpyDeviceToHost, ex->stream));
    HIP_TRY(hipStreamSynchronize(ex->stream));
    std::memcpy(n_per_frame, ex->h_n, sizeof(int) * batch);
    rc = check_status(ex, batch);
    if (rc != ORBX_OK) return rc;
    int overflow = 0;
    for (int b = 0; b < batch; b++) {
        const int n = n_per_frame[b] < cap ? n_per_frame[b] : cap;
        if (n_per_frame[b] > cap) overflow = 1;
        if (n > 0) {
            if (kps)
                HIP_TRY(hipMemcpyAsync(ex->h_kps + (size_t)b * cap, ex->d_kps + (size_t)b * cap,
                                       sizeof(orbx_keypoint) * n, hipMemcpyDeviceToHost, ex->stream));
            if (desc)
                HIP_TRY(hipMemcpyAsync(ex->h_desc + (size_t)b * cap * 32, ex->d_desc + (size_t)b * cap * 32,
                                       (size_t)n * 32, hipMemcpyDeviceToHost, ex->stream));
        }
    }
    HIP_TRY(hipStreamSynchronize(ex->stream));
    for (int b = 0; b < batch; b++) {
        const int n = n_per_frame[b] < cap ? n_per_frame[b] : cap;
        if (n <= 0) continue;
        if (kps) std::memcpy(kps + (size_t)b * cap, ex->h_kps + (size_t)b * cap, sizeof(orbx_keypoint) * n);
        if (desc) std::memcpy(desc + (size_t)b * cap * 32, ex->h_desc + (size_t)b * cap * 32, (size_t)n * 32);
    }
    return overflow ? fail(ORBX_ERR_CAPACITY, "more keypoints than cap") : ORBX_OK;
}

int orbx_extract(orbx_extractor* ex, const uint8_t* img, int width, int height, size_t stride, orbx_keypoint* kps,
                 uint8_t* desc, int cap, int* n_out) {
    if (!ex || !n_out) return fail(ORBX_ERR_ARG, "bad argument");
    if (!img || width <= 0 || height <= 0) return ORBX_EMPTY;
    const uint8_t* imgs[1] = {img};
    return orbx_extract_batch(ex, 1, imgs, width, height, stride, kps, desc, cap, n_out);
}

int orbx_pyramid_level_device(orbx_extractor* ex, int frame, int level, const uint8_t** d_ptr, size_t* pitch,
                              int* w, int* h) {
    if (!ex || !ex->have_pyramid) return fail(ORBX_ERR_STATE, "no extraction yet");
    if (frame < 0 || frame >= ex->last_batch || level < 0 || level >= ex->plan.L) return fail(ORBX_ERR_ARG, "range");
    const LevelGeom& g = ex->plan.lv[level];
    if (level == 0 && ex->l0) {  // level 0 read in place: the caller's frame
        if (d_ptr) *d_ptr = ex->l0 + (size_t)frame * ex->l0_fp;
        if (pitch) *pitch = ex->l0_pitch;
    } else {
        if (d_ptr) *d_ptr = ex->db.pyr + (size_t)frame * ex->plan.pyr_frame_bytes + g.off;
        if (pitch) *pitch = (size_t)g.pitch;
    }
    if (w) *w = g.w;
    if (h) *h = g.h;
    return ORBX_OK;
}

int orbx_pyramid_level(orbx_extractor* ex, int frame, int level, uint8_t* dst, size_t dst_stride, int* w, int* h) {
    const uint8_t* src = nullptr;
    size_t pitch = 0;
    int lw = 0, lh = 0;
    int rc = orbx_pyramid_level_device(ex, frame, level, &src, &pitch, &lw, &lh);
    if (rc != ORBX_OK) return rc;
    if (w) *w = lw;
    if (h) *h = lh;
    if (!dst) return ORBX_OK;
    if (dst_stride < (size_t)lw) return fail(ORBX_ERR_ARG, "dst_stride");
    HIP_TRY(hipSetDevice(ex->device));
    HIP_TRY(hipMemcpy2DAsync(dst, dst_stride, src, pitch, lw, lh, hipMemcpyDeviceToHost, ex->stream));
    HIP_TRY(hipStreamSynchronize(ex->stream));
    return ORBX_OK;
}

int orbx_hamming(const uint8_t* a32, const uint8_t* b32) {
    if (!a32 || !b32) return fail(ORBX_ERR_ARG, "null descriptor");
    int d = 0;
    for (int i = 0; i < 4; i++) {
        uint64_t x, y;
        std::memcpy(&x, a32 + 8 * i, 8);
        std::memcpy(&y, b32 + 8 * i, 8);
        d += __builtin_popcountll(x ^ y);
    }
    return d;
}

int orbx_hamming_matrix_device(const uint8_t* d_a, int na, const uint8_t* d_b, int nb, int32_t* d_dist,
                               void* stream) {
    if (na < 0 || nb < 0 || (na && !d_a) || (nb && !d_b) || (na && nb && !d_dist))
        return fail(ORBX_ERR_ARG, "bad argument");
    hipError_t e = launch_hamming_matrix(d_a, na, d_b, nb, d_dist, (hipStream_t)stream);
    return e == hipSuccess ? ORBX_OK : hip_fail(e, "hamming_matrix");
}

int orbx_window_match_device(const uint8_t* d_qdesc, int nq, const uint8_t* d_tdesc, const int32_t* d_tlevel,
                             const int32_t* d_cand_off, const int32_t* d_cand, int tie_last, int32_t* d_best_idx,
                             int32_t* d_best_dist, int32_t* d_best_level, int32_t* d_second_dist,
                             int32_t* d_second_level, void* stream) {
    if (nq < 0) return fail(ORBX_ERR_ARG, "nq");
    if (nq == 0) return ORBX_OK;
    if (!d_qdesc || !d_cand_off || !d_best_idx || !d_best_dist || !d_best_level || !d_second_dist || !d_second_level)
        return fail(ORBX_ERR_ARG, "null buffer");
    hipError_t e = launch_window_match(d_qdesc, nq, d_tdesc, d_tlevel, d_cand_off, d_cand, tie_last, d_best_idx,
                                       d_best_dist, d_best_level, d_second_dist, d_second_level, (hipStream_t)stream);
    return e == hipSuccess ? ORBX_OK : hip_fail(e, "window_match");
}

int orbx_window_match(int device, const uint8_t* qdesc, int nq, const uint8_t* tdesc, int nt, const int32_t* tlevel,
                      const int32_t* cand_off, const int32_t* cand, int tie_last, int32_t* best_idx,
                      int32_t* best_dist, int32_t* best_level, int32_t* second_dist, int32_t* second_level) {
    if (nq < 0 || nt < 0 || !cand_off) return fail(ORBX_ERR_ARG, "bad argument");
    if (nq == 0) return ORBX_OK;
    const int ncand = cand_off[nq];
    for (int i = 0; i < ncand; i++)
        if (cand[i] < 0 || cand[i] >= nt) return fail(ORBX_ERR_ARG, "candidate index out of range");
    HIP_TRY(hipSetDevice(device));
    uint8_t *dq = nullptr, *dt = nullptr;
    int32_t *dl = nullptr, *doff = nullptr, *dc = nullptr, *dout = nullptr;
    auto cleanup = [&]() {
        void* ps[] = {dq, dt, dl, doff, dc, dout};
        for (void* p : ps)
            if (p) (void)hipFree(p);
    };
    hipError_t e = hipSuccess;
    do {
        if ((e = dalloc(&dq, (size_t)nq * 32)) != hipSuccess) break;
        if ((e = dalloc(&dt, (size_t)nt * 32)) != hipSuccess) break;
        if ((e = dalloc(&dl, (size_t)nt)) != hipSuccess) break;
        if ((e = dalloc(&doff, (size_t)nq + 1)) != hipSuccess) break;
        if ((e = dalloc(&dc, (size_t)ncand)) != hipSuccess) break;
        if ((e = dalloc(&dout, (size_t)nq * 5)) != hipSuccess) break;
        if ((e = hipMemcpy(dq, qdesc, (size_t)nq * 32, hipMemcpyHostToDevice)) != hipSuccess) break;
        if (nt && (e = hipMemcpy(dt, tdesc, (size_t)nt * 32, hipMemcpyHostToDevice)) != hipSuccess) break;
        if (nt && tlevel && (e = hipMemcpy(dl, tlevel, sizeof(int32_t) * nt, hipMemcpyHostToDevice)) != hipSuccess) break;
        if ((e = hipMemcpy(doff, cand_off, sizeof(int32_t) * (nq + 1), hipMemcpyHostToDevice)) != hipSuccess) break;
        if (ncand && (e = hipMemcpy(dc, cand, sizeof(int32_t) * ncand, hipMemcpyHostToDevice)) != hipSuccess) break;
        e = launch_window_match(dq, nq, dt, tlevel ? dl : nullptr, doff, dc, tie_last, dout, dout + nq, dout + 2 * nq,
                                dout + 3 * nq, dout + 4 * nq, nullptr);
        if (e != hipSuccess) break;
        std::vector<int32_t> h((size_t)nq * 5);
        if ((e = hipMemcpy(h.data(), dout, sizeof(int32_t) * nq * 5, hipMemcpyDeviceToHost)) != hipSuccess) break;
        std::memcpy(best_idx, h.data(), sizeof(int32_t) * nq);
        std::memcpy(best_dist, h.data() + nq, sizeof(int32_t) * nq);
        std::memcpy(best_level, h.data() + 2 * nq, sizeof(int32_t) * nq);
        std::memcpy(second_dist, h.data() + 3 * nq, sizeof(int32_t) * nq);
        std::memcpy(second_level, h.data() + 4 * nq, sizeof(int32_t) * nq);
    } while (0);
    cleanup();
    return e == hipSuccess ? ORBX_OK : hip_fail(e, "orbx_window_match");
}

}  // extern "C"
