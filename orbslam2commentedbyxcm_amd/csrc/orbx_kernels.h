// orbx_kernels.h -- launch interface of the extraction kernels (orbx_extract.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "orbx.h"
#include "orbx_geometry.h"
#include "orbx_match_types.h"

namespace orbx {

// Device-resident buffers for one extractor configuration and batch capacity.
struct DeviceBuffers {
    int batch_cap = 0;
    LevelGeom* lv = nullptr;         // [L]
    CellGeom* cells = nullptr;       // [ncells]
    int16_t* rtab = nullptr;         // resize tables
    uint8_t* pyr = nullptr;          // [B][pyr_frame_bytes] image pyramid (level ROIs)
    uint8_t* blur = nullptr;         // [B][pyr_frame_bytes] Gaussian-blurred levels
    uint8_t* score = nullptr;        // [B][pyr_frame_bytes] FAST strength map M per level
    uint32_t* slots = nullptr;       // [B][slots_per_frame] packed FAST keypoints per cell
    int* cell_count = nullptr;       // [B][ncells]
    uint32_t* keys = nullptr;        // [B][keys_per_frame] packed candidates per level
    int* key_node = nullptr;         // [B][keys_per_frame] octree node of each candidate
    uint32_t* kept = nullptr;        // [B][kept_per_frame] kept keypoints (octree list order)
    int* kept_count = nullptr;       // [B][L]
    uint16_t* dt_list = nullptr;     // [B][kept_per_frame] kept slots listed tile after tile (k_describe_tiles)
    uint32_t* dt_tile = nullptr;     // [B][tiles_total] per level tile: list start << 16 | count
    int* status = nullptr;           // [B] error flags
    unsigned long long* oct_stamps = nullptr;  // [B][L][16] k_octree phase stamps (ORBX_OCT_STAMPS)
};

// Kernel status bits (DeviceBuffers::status)
enum : int { kStatusNodeOverflow = ORBX_STATUS_NODE_OVERFLOW, kStatusIterations = ORBX_STATUS_ITERATIONS };

// The pyramid an extractor kept from its last extraction (mvImagePyramid, ORBextractor.h:162):
// frame f's level l ROI starts at base + f * frame_bytes + off[l], rows pitch[l] bytes apart.
struct PyrView {
    const uint8_t* base = nullptr;
    long long frame_bytes = 0;
    int nframes = 0;           // frames of the last extraction
    int W = 0, H = 0, L = 0;
    long long off[kMaxLevels];
    int pitch[kMaxLevels], w[kMaxLevels], h[kMaxLevels];
    float scale[kMaxLevels], inv_scale[kMaxLevels];
    int device = 0;
    hipStream_t stream = nullptr;  // stream of the last extraction
    // level 0 read in place (orbx_extractor_set_level0_in_place): frame f's level 0 is the
    // caller's frame at l0 + f * l0_fp, rows l0_pitch apart (null: level 0 is in base)
    const uint8_t* l0 = nullptr;
    long long l0_fp = 0;
    int l0_pitch = 0;
};
// Fills `v` for extractor `ex` (ORBX_ERR_STATE before any extraction, and, unless
// allow_l0 -- a reader that takes level 0 from v->l0 --, after an in-place extraction).
int extractor_pyramid(orbx_extractor* ex, PyrView* v, bool allow_l0 = false);

constexpr int kStages = 6;
extern const char* const kStageNames[kStages];

// Pattern + umax into __constant__ memory (idempotent).
hipError_t upload_constants(const OrbParams& prm);

// Enqueue the whole extraction of `batch` device frames on `stream`.
// kps: orbx_keypoint[batch*cap], desc: uint8[batch*cap*32], n_per_frame: int[batch].
// ev (nullable) holds kStages+1 events recorded between the stages.  status_out (nullable,
// e.g. host-mapped memory): the describe kernel copies each frame's octree status word there
// beside its count, so a host call learns both without a separate read-back.
hipError_t launch_extract(const Plan& plan, const DeviceBuffers& db, int batch, const uint8_t* d_imgs,
                          size_t frame_pitch, size_t stride, void* kps, uint8_t* desc, int cap,
                          int* n_per_frame, hipStream_t stream, hipEvent_t* ev,
                          hipEvent_t stage_ev = nullptr, int stage_after = 0, bool l0_in_place = false,
                          int* status_out = nullptr);

// dist[i*nb+j] = Hamming(a_i, b_j)
hipError_t launch_hamming_matrix(const uint8_t* a, int na, const uint8_t* b, int nb, int32_t* dist,
                                 hipStream_t stream);

hipError_t launch_proj_search(const ProjProblem* d_probs, int nprob, const ProjParams& P, unsigned long long* scratch,
                              const long long* d_scratch_off, int max_n, int max_nq, hipStream_t stream,
                              bool small = false, bool tiny = false, bool lean = false,
                              unsigned char* split_grids = nullptr);

// k_seq_grid + k_seq_score + k_seq_commit: the split form of launch_proj_search for the
// batched sequence matcher (grids: nprob x seq_grid_bytes(cap) bytes of device memory).
// cap: keypoints per problem (the grids); qcap: queries per problem (0: cap).  stage_*
// (one problem only): k_stage_copy first copies stage_bytes (a multiple of 16) from
// device-visible pinned host memory to stage_dst -- the call's inputs, d_probs among them
size_t seq_grid_bytes(int cap, int noct);
// k_stage_copy: bytes (a multiple of 16, 16-byte aligned ends) between device memory and
// device-visible (mapped) pinned host memory, by the GPU's own loads and stores (many
// workgroups) instead of a DMA copy -- for the small per-call copies of the host calls
hipError_t launch_stage_copy(const void* src, void* dst, size_t bytes, hipStream_t stream);
hipError_t launch_seq_split(const ProjProblem* d_probs, int nprob, const ProjParams& P, unsigned char* grids,
                            int cap, unsigned long long* scratch, const long long* d_scratch_off, hipStream_t stream,
                            int qcap = 0, int replay_rt = 0, const void* stage_src = nullptr,
                            void* stage_dst = nullptr, size_t stage_bytes = 0);

hipError_t launch_seq_build(const SeqArgs& A, int npairs, ProjQuery* queries, ProjProblem* probs,
                            long long* scratch_off, hipStream_t stream);
// k_local_build: Tracking::SearchLocalPoints' problem per frame (one workgroup each)
hipError_t launch_local_build(const LocalArgs& A, int batch, ProjQuery* queries, uint8_t* qdesc, ProjProblem* probs,
                              long long* scratch_off, hipStream_t stream);

hipError_t launch_triangulation(const TriProblem* d_probs, int nprob, unsigned long long* scratch, int max_n2,
                                int max_nq, hipStream_t stream);
// k_tri_setup (queries + problems from the keyframe tables) then k_triangulation
hipError_t launch_triangulation_batch(const TriBatch& tb, unsigned long long* scratch, hipStream_t stream);

hipError_t launch_stereo(const StereoBatch& sb, int batch, hipStream_t stream);
hipError_t launch_bow(const BowProblem* d_prob, int n2, int nitems, hipStream_t stream);
hipError_t launch_init(const InitProblem* d_prob, int n1, int n2, int nq, hipStream_t stream);
hipError_t launch_window_best(const BestProblem* d_prob, int nq, hipStream_t stream);
hipError_t launch_distinctive(int nmp, const int32_t* off, const uint8_t* desc, int32_t* best, uint8_t* out_desc,
                              hipStream_t stream);

hipError_t launch_window_match(const uint8_t* qdesc, int nq, const uint8_t* tdesc, const int32_t* tlevel,
                               const int32_t* cand_off, const int32_t* cand, int tie_last,
                               int32_t* best_idx, int32_t* best_dist, int32_t* best_level,
                               int32_t* second_dist, int32_t* second_level, hipStream_t stream);

}  // namespace orbx
