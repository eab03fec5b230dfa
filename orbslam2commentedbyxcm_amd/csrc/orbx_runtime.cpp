// orbx_runtime.cpp -- library-wide runtime state: the thread-local last-error string
// (orbx_last_error), the unload flag (DESIGN.md §1 "Teardown"), and the alternative kernel
// forms and diagnostics switches.
//
// The product reads no environment.  A form other than the measured default (each gives
// the same results; the GPU tests run them) is selected only through orbx_debug_set, by the
// tests and the A/B tools; the ORBX_* environment variables of earlier rounds are read only
// by a debug build (-DORBX_DEBUG=1: python -m orbslam2commentedbyxcm_amd.build --variant
// debug -DORBX_DEBUG=1), where they take precedence over nothing but the defaults.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>

#include "orbx.h"
#include "orbx_error.h"

namespace orbx {
namespace {

thread_local std::string g_last_error;
std::atomic<bool> g_unloading{false};

// runs from the C runtime's exit / dlclose teardown of this library -- before that of the
// HIP runtime it links against (dependents are finalised first)
__attribute__((destructor)) void orbx_on_unload() { g_unloading.store(true); }

struct Knob {
    const char* name;  // orbx_debug_set name
    const char* env;   // the debug build's environment variable
};

// the switches, by index (orbx_error.h: enum Tune)
constexpr Knob kKnobs[] = {
    {"pz_seg", "ORBX_PZ_SEG"},                 // pyramid levels per k_pyramid launch (0: one launch)
    {"pz_byte", "ORBX_PZ_BYTE"},               // k_pyramid's byte-read form
    {"desc_tiles", "ORBX_DESC_TILES"},         // tile-major k_describe_tiles (measured slower)
    {"extract_dma", "ORBX_EXTRACT_DMA"},       // single host call through DMA copies, not mapped memory
    {"replay_threads", "ORBX_REPLAY_THREADS"}, // replay workgroup width (64 .. 1024)
    {"dup_stage", "ORBX_DUP_STAGE"},           // launch extraction stage k twice (marginal-cost pricing)
    {"oct_stamps", "ORBX_OCT_STAMPS"},         // k_octree phase stamps (diagnostics)
    {"call_stamps", "ORBX_CALL_STAMPS"},       // single matcher calls' phase stamps (diagnostics)
    {"match_stamps", "ORBX_MATCH_STAMPS"},     // batched matcher phase stamps (diagnostics)
};
constexpr int kNumKnobs = sizeof(kKnobs) / sizeof(kKnobs[0]);
std::atomic<int> g_set[kNumKnobs];      // orbx_debug_set values
std::atomic<bool> g_has[kNumKnobs];     // ... and whether one is set

}  // namespace

void set_last_error(const std::string& msg) { g_last_error = msg; }
bool unloading() { return g_unloading.load(); }

int tuning(Tune k, int dflt) {
    const int i = (int)k;
    if (i < 0 || i >= kNumKnobs) return dflt;
    if (g_has[i].load(std::memory_order_relaxed)) return g_set[i].load(std::memory_order_relaxed);
#if ORBX_DEBUG
    if (const char* e = std::getenv(kKnobs[i].env)) return std::atoi(e);
#endif
    return dflt;
}

const char* debug_env(const char* name) {
#if ORBX_DEBUG
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

}  // namespace orbx

extern "C" const char* orbx_last_error(void) { return orbx::g_last_error.c_str(); }

extern "C" int orbx_debug_set(const char* name, int value) {
    if (!name) {  // every switch back to its default
        for (int i = 0; i < orbx::kNumKnobs; i++) orbx::g_has[i].store(false);
        return ORBX_OK;
    }
    for (int i = 0; i < orbx::kNumKnobs; i++)
        if (!std::strcmp(name, orbx::kKnobs[i].name)) {
            orbx::g_set[i].store(value);
            orbx::g_has[i].store(value >= 0);
            return ORBX_OK;
        }
    orbx::set_last_error(std::string("unknown switch: ") + name);
    return ORBX_ERR_ARG;
}
