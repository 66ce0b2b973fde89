// Persistent multi-universe trainer: host side (row shapes, shape classes, the LDS plan dispatch) and the
// general (plan 0) kernels. Device code in universes_kern.h; plans 1 and 2 in universes_p1.hip / _p2.hip.
#include "universes_kern.h"

namespace pt {

Shape pick_universe_shape(int64_t D, bool wide) {
    const int VEC = D % 4 == 0 ? 4 : 1;
    const int64_t chunks = (D + VEC - 1) / VEC;
    const int64_t per_lane = wide ? universe_chunks_per_lane(0, VEC) : universe_chunks_per_lane(1, VEC);
    int G = 2;
    while (G < 64 && (int64_t)G * per_lane < chunks) G <<= 1;
    int KCH = 1;
    while ((int64_t)G * KCH < chunks) KCH <<= 1;
    if (dev::exact_kch_shape(G, VEC)) KCH = (int)((chunks + G - 1) / G);   // no power-of-two padding (universes_kern.h)
    return Shape{G, VEC, KCH};
}

int universe_shape_id(int64_t D, int model) {
    if (D <= 0) return -1;
    // TransE (few live rows per step) takes the wide shapes: twice the lane groups, half the rounds of a
    // step's positives (PT_UNI_NARROW=1: the narrow ones)
    static const bool narrow = [] {
        const char *v = pt_tuning_env("PT_UNI_NARROW");
        return v && atoi(v) != 0;
    }();
    const Shape s = pick_universe_shape(D, model == 0 && !narrow);
    // (a shape its class kernel does not compile would leave the universe untrained: unsupported instead)
#define PT_USUP(ID_, G_, V_, K_) \
    if (s.G == G_ && s.VEC == V_ && s.KCH == K_) return dev::shape_reachable(model, G_, V_, K_) ? ID_ : -1;
    PT_USHAPES(PT_USUP)
#undef PT_USUP
    return -1;
}

bool universe_shape_supported(int64_t D, int model) { return universe_shape_id(D, model) >= 0; }

// shape class of a row shape (one kernel per class)
int universe_shape_class(int shape) {
#define PT_UCLS(ID_, G_, V_, K_) \
    if (shape == ID_) return PT_UCLASS(V_, K_);
    PT_USHAPES(PT_UCLS)
#undef PT_UCLS
    return 1;
}

// lane groups of a universe workgroup for a shape (positives of a step processed concurrently)
int universe_shape_groups(int shape, int model) {
#define PT_UGPB(ID_, G_, V_, K_) \
    if (shape == ID_) return universe_class_threads(model, PT_UCLASS(V_, K_)) / G_;
    PT_USHAPES(PT_UGPB)
#undef PT_UGPB
    return 1;
}

// padded row length of a row shape (lanes x floats per lane: the floats a lane group touches per row)
int universe_shape_row_slots(int shape) {
#define PT_URS(ID_, G_, V_, K_) \
    if (shape == ID_) return G_ * V_ * K_;
    PT_USHAPES(PT_URS)
#undef PT_URS
    return 1;
}

// the LDS plan the launch configuration amounts to (universe_run's PLAN): 1 and 2 are compiled apart with
// their choices fixed, anything else takes the general kernel
static int universe_plan(const UniverseLaunch &cfg) {
    if (!cfg.contrib || cfg.pchunk <= 0 || cfg.agent_fence) return 0;
    if (cfg.rel_list) return 2;
    return cfg.lds_relgrad && cfg.lds_flags ? 1 : 0;
}

hipError_t launch_universes(const UniverseDev *d_us, int64_t n, int *counter, int cls, int64_t cus, int model,
                            int p_norm, int norm_flag, int opt, int64_t neg, int bern, int filter,
                            const UniverseLaunch &cfg, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    switch (universe_plan(cfg)) {
        case 1:
            return launch_universes_plan<1>(d_us, n, counter, cls, cus, model, p_norm, norm_flag, opt, neg, bern, filter,
                                            cfg, st);
        case 2:
            return launch_universes_plan<2>(d_us, n, counter, cls, cus, model, p_norm, norm_flag, opt, neg, bern, filter,
                                            cfg, st);
        default:
            return launch_universes_plan<0>(d_us, n, counter, cls, cus, model, p_norm, norm_flag, opt, neg, bern, filter,
                                            cfg, st);
    }
}

}  // namespace pt
