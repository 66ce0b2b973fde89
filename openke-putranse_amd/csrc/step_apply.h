// Host interface of the fused step + apply kernel (step_apply.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace pt {

// state of the fused step + apply beyond the counting-sort workspace (zero between steps: every row's last
// arriver re-zeroes its arrival word and its gradient row)
struct FusedRows {
    float *gent = nullptr, *grel = nullptr;   // [rows][dp] gradient rows of the positives' h / t and r
    uint64_t *arrive = nullptr;               // [E + R] arrivals of each row this step (entities, then relations
                                              // at CsrWork::rel_base)
    int32_t dp = 0;                           // row stride of gent / grel / the contribution rows, in floats
};

// padded row stride (floats): a multiple of 32, so every row starts on a 128-B line and owns its lines
int64_t step_apply_row_stride(int64_t dim);
// whether the fused kernel takes this TransE configuration (float4 rows of 33-256 chunks, offsets in 31 bits)
bool step_apply_supported(const StepParams &P, int64_t bs, int64_t neg);
// one training step of the call `v` (csr_view), the tables updated in place; the step's loss partials go to
// v.lpart (launch_loss_calls turns a chunk's into losses)
hipError_t launch_step_apply(const StepParams &P, const CsrWork &v, const FusedRows &fr, hipStream_t st);
// losses of `calls` consecutive calls from their partials ([calls][bs]): loss[i] = (or +=) inv_count * sum + margin
hipError_t launch_loss_calls(const float *lpart, int64_t bs, int64_t calls, float inv_count, float margin, float *loss,
                             int assign, hipStream_t st);

}  // namespace pt
