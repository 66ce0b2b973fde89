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
    float *contrib;                                 // [bs*(4+neg)][dim] gradient-row contributions
    float *ord;                                     // reference-order mode: [4][seq][dim] per-slot gradient rows
    float *losses;                                  // [epochs] Trainer.run's per-epoch loss sum (or null)
    uint64_t *prof;                                 // null, or [64]: cycles (presample, A, B), steps, bs, dim, E, 0, stamps
    int64_t threads, bs, nbatches, epochs, dim;
    float lr, margin;
    int32_t shape;                                  // universe_shape_id(dim)
};

// A team universe's exchange state (universes_team.h), beside its UniverseDev (kept apart: the class kernels hold
// a register copy of their descriptor, whose size their SGPR spills follow)
struct TeamDev {
    float *part;                                    // [w][rel][dim] relation partials, [w][epochs] loss partials,
                                                    // [w] the members' XCD ids
    uint32_t *sync;                                 // arrival counter (zeroed before each launch)
    uint32_t *err;                                  // the set's error word (a bounded poll ran out)
    int32_t w;                                      // members
};

// workgroup size of each (model, shape class) kernel. TransE's narrow classes (<= 8 floats per lane) run 1,024
// threads (16 waves, 4 per SIMD, 128 VGPRs: twice the lane groups, so a step's positives take half the rounds
// and twice the waves hide each other's latency; measured C3 57.4 -> 52.5 ms, its longest universe 135 -> 100
// Mcycles); the 16-float class and TransH (whose step keeps more rows live: at 128 VGPRs it spills, C5 37 -> 89
// ms) keep 512 threads at 256 VGPRs
#ifndef PT_UNI_NT
#define PT_UNI_NT 1024
#endif
constexpr int universe_class_threads(int model, int cls) { return model == 0 && cls < 2 ? PT_UNI_NT : 512; }
// workgroup size of a hot single-shape kernel for lane groups of G lanes: PT_UNI_HOT_WIDE_NT for the wide rows
// (G >= 32: C4's D = 200 on 32 lanes x 8 floats), the class size otherwise
#ifndef PT_UNI_HOT_WIDE_NT
#define PT_UNI_HOT_WIDE_NT 1024
#endif
constexpr int universe_hot_threads(int G) { return G >= 32 ? PT_UNI_HOT_WIDE_NT : PT_UNI_NT; }
// class ids from kUniHotBase on: a "hot" class-1 shape (id - kUniHotBase) run by a kernel compiled for that shape
// alone (its own register allocation; see pt_universe_set_create)
constexpr int kUniHotBase = 64;
// class ids from kUniTeamBase on: universes of shape (id - kUniTeamBase) trained by teams of workgroups
// (universes_team.h), one launch per shape
constexpr int kUniTeamBase = 128;

// launch configuration of one group of universes (host-chosen for the largest universe of the group)
struct UniverseLaunch {
    int threads = 512;          // workgroup size
    int64_t list_cap = 1;       // LDS work-list entries (>= bs * (4 + neg))
    int lds_flags = 0;          // touched-row flags in LDS instead of the global flag arrays
    int contrib = 0;            // entity gradients as LDS-linked contribution slots (needs head[E] + next[ccap])
    int64_t pchunk = 0;         // batches drawn into LDS at a time (0: sample inside each step)
    int lds_relgrad = 0;        // relation / norm_vector gradient rows in LDS (R x D floats, x2 for TransH)
    int rel_list = 0;           // relation / norm_vector rows as contribution lists (when their rows do not fit)
    int agent_fence = 1;        // agent-scope fences around the phase barriers (global atomics in use)
    int64_t lds_bytes = 0;      // dynamic LDS per workgroup
};

// lane-group shape of the universe kernel for dim D (narrower groups than pick_shape) and its id in
// the kernel's shape switch (-1: unsupported)
// chunks of VEC floats per lane of a universe row shape: 8 floats per lane for TransE's scalar rows (wide:
// twice the lane groups, half the rounds of a step's positives), 4 for TransH's; float4 rows 2 chunks (8 floats)
// for both. (r04, same box: float4 TransE rows at 8 instead of 16 floats per lane moved them from the 512-thread
// 16-float class kernel, whose CU share finished last, to the 1,024-thread 8-float one: C3 52.5 -> 40.2 ms,
// C4 105.8 -> 104.0 ms; only TransE rows over 512 floats still take the 16-float class.)
constexpr int universe_chunks_per_lane(int model, int vec) { return vec == 4 ? 2 : (model == 0 ? 8 : 4); }
Shape pick_universe_shape(int64_t D, bool wide);
int universe_shape_id(int64_t D, int model);
bool universe_shape_supported(int64_t D, int model);

// the n universes of one shape class (d_us[0..n), longest first) in one persistent launch of that
// class's kernel over `cus` CUs' worth of workgroups: workgroups pull universes from *counter (device
// int, reset by the launch)
hipError_t launch_universes(const UniverseDev *d_us, int64_t n, int *counter, int cls, int64_t cus, int model,
                            int p_norm, int norm_flag, int opt, int64_t neg, int bern, int filter,
                            const UniverseLaunch &cfg, hipStream_t st);
int universe_shape_class(int shape);
// team universes (universes_team.h): whether a shape has a team kernel (TransE, 8-float class), the dynamic LDS of
// its launch, and the launch over `grid` workgroups (map: [grid][2] universe index into d_us, member or -1)
bool universe_team_shape(int shape, int model);
int64_t universe_team_lds_bytes(int64_t list_cap, int64_t rel, int64_t ent, int64_t slots, int64_t pchunk,
                                int64_t seq, int64_t rel_step, int64_t dim);
hipError_t launch_universes_team(const UniverseDev *d_us, const TeamDev *d_teams, const int32_t *d_map, int64_t grid,
                                 int shape, int p_norm, int norm_flag, int opt, int64_t neg, int bern, int filter,
                                 const UniverseLaunch &cfg, hipStream_t st);
int universe_shape_groups(int shape, int model);
int universe_shape_row_slots(int shape);

}  // namespace pt
