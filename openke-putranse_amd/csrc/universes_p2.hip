// Universe kernels of LDS plan 2 (universe_run), compiled apart from the others (build parallelism).
#include "universes_kern.h"

namespace pt {
template hipError_t launch_universes_plan<2>(const UniverseDev *, int64_t, int *, int, int64_t, int, int, int, int,
                                              int64_t, int, int, const UniverseLaunch &, hipStream_t);
}  // namespace pt
