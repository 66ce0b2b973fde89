// Measurement-build switches. `make TUNING=1` defines PT_TUNING: the environment variables the sources
// read through pt_tuning_env() (PT_STEP_*, PT_APPLY_*, PT_PART_*, PT_CSR, PT_UNI_*, PT_LP_BATCH_MB) then pick
// kernel shapes, placements and ablations for A/B timing, and PT_ABLATE(bits, mask) enables the timing-only
// ablations whose results are wrong (StepParams::dbg, CsrWork::dbg). The product build ignores the
// environment entirely: pt_tuning_env() returns null and PT_ABLATE() is a constant false, so no variable
// left in a user's shell can change a kernel's path or its results, and the ablation branches compile away.
#pragma once
#include <cstdlib>

#ifdef PT_TUNING
inline const char *pt_tuning_env(const char *name) { return std::getenv(name); }
#define PT_ABLATE(bits, mask) (((bits) & (mask)) != 0)
#else
inline const char *pt_tuning_env(const char *) { return nullptr; }
#define PT_ABLATE(bits, mask) false
#endif
