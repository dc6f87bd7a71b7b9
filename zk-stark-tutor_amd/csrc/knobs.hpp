// Kernel-plan constants and where they may come from (VERDICT r05 "Next round" 7).
//
// Product builds compile the measured defaults in and read NO environment variable for the kernel
// plan: a caller's environment cannot switch a tile size, a tree layout or a stream priority.  The
// library's only runtime environment settings are documented in INTEGRATION.md §9 (pool cap,
// domain cache, and the communicator's FRI hand-over / algebra sharding / deadline); the test
// switches that compare equivalent paths are explicit calls (sg_ctx_set_option).
//
// An A/B build (make EXTRA=-DSG_AB_KNOBS=1 BUILD=build_ab OUT=starkgpu/libstarkgpu_ab.so) reads
// SG_<NAME> for every SG_KNOB below, once per process, and initializes each context's options from
// SG_AIR_GENERIC / SG_GEO_DECIMATE / SG_LEAN_TREES / SG_STREAM_NO_PIN / SG_DIST_WORLD1_SHARDED:
// the alternate-paths suite (tools/gpu_alt_paths.sh) and the A/B runner (tools/ab.sh) load it
// through SG_LIB_PATH.
#pragma once

#ifndef SG_AB_KNOBS
#define SG_AB_KNOBS 0
#endif

namespace sg {
// A/B builds: SG_<name> from the environment (atoi), else `def`
int ab_knob(const char* name, int def);
}  // namespace sg

#if SG_AB_KNOBS
#define SG_KNOB(NAME, DEF) ::sg::ab_knob("SG_" #NAME, (DEF))
#else
#define SG_KNOB(NAME, DEF) (DEF)
#endif
