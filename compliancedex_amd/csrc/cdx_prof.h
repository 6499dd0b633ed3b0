// Optional per-stage HIP-event timing of the closure pipeline (bench.py reads it through
// cdx_profile_enable / cdx_profile_read).  Events are recorded on the launch stream
// around each kernel of the enabled stages, so they time exactly what runs; disabled by default.
#pragma once
#include <hip/hip_runtime.h>

namespace cdx {
enum ProfStage { PROF_QUERIES = 0, PROF_GPIS_MEAN = 1, PROF_GPIS_STD = 2, PROF_COST = 3, PROF_GPIS_GRAD = 4, PROF_SCREEN = 5,
                 PROF_STAGES = 6 };
void prof_mark(int stage, bool begin, hipStream_t s);  // defined in cdx_closure.hip
}  // namespace cdx
