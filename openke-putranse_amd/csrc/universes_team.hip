// Team-universe kernels (universes_team.h), one per 8-float-class TransE row shape, compiled apart.
#include "universes_team.h"

namespace pt {

bool universe_team_shape(int shape, int model) {
    if (model != 0) return false;
#define PT_UTS(ID_, G_, V_, K_) \
    if (shape == ID_) return PT_UCLASS(V_, K_) == 1 && dev::shape_reachable(0, G_, V_, K_);
    PT_USHAPES(PT_UTS)
#undef PT_UTS
    return false;
}

// universe_run_team's LDS carve (int32 units, each region rounded to 4): work list, own rows, entity list heads,
// relation map, the step's relations, slot links, presampled batches, the step relations' gradient rows
int64_t universe_team_lds_bytes(int64_t list_cap, int64_t rel, int64_t ent, int64_t slots, int64_t pchunk, int64_t seq,
                                int64_t rel_step, int64_t dim) {
    auto a4 = [](int64_t v) { return (v + 3) & ~int64_t(3); };
    return 4 * (2 * a4(list_cap) + a4(ent) + a4(rel) + a4(rel_step) + a4(slots) + 3 * pchunk * seq + rel_step * dim);
}

namespace {
template <int ID, int G, int VEC, int KCH>
hipError_t launch_team_shape(const UniverseDev *d_us, const TeamDev *d_teams, const int32_t *d_map, int64_t grid,
                             int p_norm, int norm_flag, int opt, int64_t neg, int bern, int filter,
                             const UniverseLaunch &cfg, hipStream_t st) {
    constexpr int NT = universe_hot_threads(G);
    auto kern = dev::k_universes_team<NT, ID, G, VEC, KCH>;
    if (cfg.lds_bytes > (64 << 10)) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)cfg.lds_bytes);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), (size_t)cfg.lds_bytes, st, d_us, d_teams, d_map, p_norm,
                       norm_flag, opt, neg, bern, filter, cfg);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_universes_team(const UniverseDev *d_us, const TeamDev *d_teams, const int32_t *d_map, int64_t grid,
                                 int shape, int p_norm, int norm_flag, int opt, int64_t neg, int bern, int filter,
                                 const UniverseLaunch &cfg, hipStream_t st) {
    if (grid <= 0) return hipSuccess;
    switch (shape) {
#define PT_UTL(ID_, G_, V_, K_)                                                                                  \
    case ID_:                                                                                                    \
        if constexpr (PT_UCLASS(V_, K_) == 1 && dev::shape_reachable(0, G_, V_, K_))                             \
            return launch_team_shape<ID_, G_, V_, K_>(d_us, d_teams, d_map, grid, p_norm, norm_flag, opt, neg, bern, \
                                                      filter, cfg, st);                                          \
        break;
        PT_USHAPES(PT_UTL)
#undef PT_UTL
        default:
            break;
    }
    return hipErrorInvalidValue;
}

}  // namespace pt
