// orbx_error.h -- thread-local last-error string shared by the ABI translation units.
#pragma once

#include <string>

namespace orbx {
void set_last_error(const std::string& msg);
// True once liborbx's own unload destructor has run (process exit, dlclose): the HIP
// runtime, which liborbx depends on and which is therefore finalised after it, may be
// going away, so the orbx_*_destroy entry points release nothing and leave the memory and
// streams to the process teardown.  DESIGN.md §1 "Teardown".
bool unloading();

// Alternative kernel forms and diagnostics switches (orbx_runtime.cpp): the value set by
// orbx_debug_set, else (debug builds only) the ORBX_* environment variable, else dflt.
enum class Tune { PzSeg, PzByte, DescTiles, ExtractDma, ReplayThreads, DupStage, OctStamps, CallStamps, MatchStamps };
int tuning(Tune k, int dflt);
// the environment variable `name` in a debug build (-DORBX_DEBUG=1), nullptr in the product
const char* debug_env(const char* name);
}
