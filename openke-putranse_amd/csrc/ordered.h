// Reference-order (deterministic) training step (ordered.hip): launch interface.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace pt {

struct UniverseDev;

// One step on an explicit batch in the reference layout (negative k of positive i at (k+1)*bs+i) with
// its scratch: score / ds [seq], per-slot gradient rows gh / gt / gr / gw [seq][dim] (gw: TransH only).
struct OrderedStep {
    int model, p_norm, norm_flag, opt;
    float lr, margin;
    int64_t ent_total, rel_total, dim;
    float *ent, *rel, *normv;
    float *ent_acc, *rel_acc, *norm_acc;
    const int64_t *h, *t, *r;
    int64_t seq, bs, neg;
    float *score, *ds;
    float *gh, *gt, *gr, *gw;
};

bool ordered_dim_supported(int64_t dim);
// loss: the step's loss is stored (assign) or added to *loss (device; may be null)
hipError_t launch_ordered_step(const OrderedStep &S, float *loss, int assign, hipStream_t st);
// dynamic LDS of the ordered universe kernel for universes of at most max_seq slots per step
int64_t ordered_universe_lds_bytes(int64_t max_seq);
// static LDS of the reference-order universe kernel (its __shared__ variables, next to the dynamic area)
hipError_t ordered_universe_static_lds(size_t *bytes);
// every universe of d_us[0..n) trained in reference order, one 256-thread workgroup per universe taken
// from *counter; each UniverseDev needs `ord` scratch of 4 * seq * dim floats
hipError_t launch_universes_ordered(const UniverseDev *d_us, int64_t n, int *counter, int64_t cus, int model,
                                    int p_norm, int norm_flag, int opt, int64_t neg, int bern, int filter,
                                    int64_t max_seq, hipStream_t st);

}  // namespace pt
