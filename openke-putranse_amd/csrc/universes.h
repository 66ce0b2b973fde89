// Device descriptor + launcher of the persistent multi-universe trainer (universes.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "graph.h"
#include "kernels.h"

namespace pt {

// One universe's training job as the kernel sees it (all pointers device memory).
struct UniverseDev {
    DeviceGraph g;                                  // universe-local training graph
    uint64_t *states;                               // [threads] LCG states (advanced in place)
    float *ent, *rel, *normv;                       // tables [E_u|R_u][dim]
    float *ent_acc, *rel_acc, *norm_acc;            // Adagrad accumulators (same shapes)
    float *gent, *grel, *gnorm;                     // gradient rows, zero between steps
    int32_t *fent, *frel, *fnorm;                   // touched-row flags, zero between steps
    float *losses;                                  // [epochs] Trainer.run's per-epoch loss sum (or null)
    int64_t threads, bs, nbatches, epochs, dim;
    float lr, margin;
};

// n universes of one row shape `s` in one launch (one workgroup each); list_cap = LDS work-list entries
// (>= bs * (4 + neg) for every universe of the launch)
hipError_t launch_universes(const UniverseDev *d_us, int64_t n, const Shape &s, int model, int p_norm, int norm_flag,
                            int opt, int64_t neg, int bern, int filter, int64_t list_cap, hipStream_t st);

}  // namespace pt
