// Persistent multi-universe trainer (PuTransE / PuTransH, BASELINE configs C3-C5).
//
// The reference trains its universes one after another, each with Trainer.run over
// epochs x nbatches tiny minibatches (Parallel_Universe_Config.py:228-258, Trainer.py:90-104); a
// universe step is ~25-100 positives, far too small for a launch per step. Here ONE workgroup owns
// ONE universe for its whole training run: every epoch and minibatch is a loop iteration inside the
// kernel, with two workgroup barriers per step that give the reference's minibatch-synchronous
// semantics (every gradient of a step sees the pre-step tables):
//
//   phase A  each lane group takes positives b = grp, grp + GPB, ... of the step: draws the positive
//            and its negatives exactly as sampling() would (per-universe LCG streams kept in LDS),
//            runs group_step (forward, MarginLoss, backward) and adds the gradient rows into the
//            universe's gradient buffer with float atomics; the first touch of a row appends it to
//            an LDS work list;
//   phase B  the lane groups walk the work list: normalize Jacobian of the pre-step row where the
//            table's gradient is in normalized space, then the Adagrad (or SGD) row update, and
//            re-zero the gradient row / flag; the sampler streams advance by the step's draws.
//
// Universes are independent, so thousands run concurrently (one per workgroup, several per CU) and
// universes of different embedding dims run as separate launches on separate streams. The tables
// stay in HBM (a universe's rows are re-read every step, so they live in L2 / Infinity Cache).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device.h"
#include "kernels.h"
#include "universes.h"

namespace pt {
namespace dev {

// release / acquire at agent scope around the workgroup barrier: stores of one phase are visible to
// loads of the next phase from any wave (L1 invalidated), independent of L1 write policy
__device__ __forceinline__ void phase_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// Gradient sink of one universe: float atomics into the gradient rows, first touch of a row appends
// (row << 2 | table) to the LDS work list.
struct UniverseSink {
    float *gent, *grel, *gnorm;
    int32_t *fent, *frel, *fnorm;
    int32_t *list;
    int *count;
    __device__ __forceinline__ void touch(int32_t *flag, int64_t row, int table) const {
        if (atomicExch(flag + row, 1) == 0) list[atomicAdd(count, 1)] = (int32_t)(row << 2) | table;
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void ent(int64_t row, const V<G, VEC, KCH> &g, int D, int lane) const {
        vatomic(g, gent + row * D, D, lane);
        if (lane == 0) touch(fent, row, 0);
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void rel(int64_t row, const V<G, VEC, KCH> &g, int D, int lane) const {
        vatomic(g, grel + row * D, D, lane);
        if (lane == 0) touch(frel, row, 1);
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void norm(int64_t row, const V<G, VEC, KCH> &g, int D, int lane) const {
        vatomic(g, gnorm + row * D, D, lane);
        if (lane == 0) touch(fnorm, row, 2);
    }
};

template <int MODEL, int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_universes(const UniverseDev *__restrict__ us, int p_norm, int norm_flag,
                                                   int opt, int64_t neg, int bern, int filter) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    extern __shared__ int32_t s_list[];
    __shared__ uint64_t s_states[64];
    __shared__ int s_count;
    __shared__ float s_loss;
    const UniverseDev U = us[blockIdx.x];
    const int tid = threadIdx.x, lane = tid % G, grp = tid / G;
    const int64_t bs = U.bs, threads = U.threads, D = U.dim;
    if (tid < threads) s_states[tid] = U.states[tid];
    StepParams P{};
    P.model = MODEL; P.p_norm = p_norm; P.norm_flag = norm_flag; P.opt = opt;
    P.lr = U.lr; P.margin = U.margin;
    P.ent_total = U.g.ent_total; P.rel_total = U.g.rel_total; P.dim = D;
    P.ent = U.ent; P.rel = U.rel; P.normv = U.normv;
    P.ent_acc = U.ent_acc; P.rel_acc = U.rel_acc; P.norm_acc = U.norm_acc;
    P.batch_size = bs; P.neg = neg;
    P.inv_count = 1.0f / (float)(bs * neg);
    const UniverseSink sink{U.gent, U.grel, U.gnorm, U.fent, U.frel, U.fnorm, s_list, &s_count};
    const int64_t dpp = 1 + 2 * neg;
    const DeviceGraph &g = U.g;
    float epoch_loss = 0.f;
    for (int64_t epoch = 0; epoch < U.epochs; ++epoch) {
        for (int64_t step = 0; step < U.nbatches; ++step) {
            if (tid == 0) {
                s_count = 0;
                s_loss = 0.f;
            }
            phase_barrier();
            // ---- phase A: sample + forward + backward of the step's positives
            for (int64_t b = grp; b < bs; b += GPB) {
                const PosDraw pd = draw_positive(g, s_states, threads, bs, b, dpp);
                const float lsum = group_step<MODEL, G, VEC, KCH>(
                    P, pd.h, pd.r, pd.t, neg,
                    [&](int64_t k, int64_t &h, int64_t &t, int64_t &r) {
                        int side;
                        const int64_t e = draw_negative(g, pd, k, bern, filter, &side);
                        h = side ? pd.h : e;
                        t = side ? e : pd.t;
                        r = pd.r;
                    },
                    sink, lane);
                if (lane == 0) atomicAdd(&s_loss, lsum);
            }
            phase_barrier();
            // ---- phase B: row updates of the touched rows
            const int n = s_count;
            for (int i = grp; i < n; i += GPB) {
                const int32_t code = s_list[i];
                const int table = code & 3;
                const int64_t row = code >> 2;
                float *w = table == 0 ? U.ent : (table == 1 ? U.rel : U.normv);
                float *acc = table == 0 ? U.ent_acc : (table == 1 ? U.rel_acc : U.norm_acc);
                float *gr = table == 0 ? U.gent : (table == 1 ? U.grel : U.gnorm);
                int32_t *fl = table == 0 ? U.fent : (table == 1 ? U.frel : U.fnorm);
                // ent rows of TransE and every rel / norm_vector row carry normalized-space gradients
                const bool jac = table == 0 ? (MODEL == 0 && norm_flag) : (table == 1 ? norm_flag != 0 : true);
                Vec x, gs, gg;
                vload(x, w + row * D, (int)D, lane);
                vload(gs, gr + row * D, (int)D, lane);
                if (jac) {
                    const float nx = sqrtf(vdot(x, x));
                    vnormalize_bwd(x, nx, gs, gg);
                } else {
                    gg = gs;
                }
                if (opt == 0) {
#pragma unroll
                    for (int j = 0; j < Vec::N; ++j) x.x[j] = x.x[j] + (-U.lr) * gg.x[j];
                } else {
                    Vec a;
                    vload(a, acc + row * D, (int)D, lane);
#pragma unroll
                    for (int j = 0; j < Vec::N; ++j) {
                        a.x[j] = a.x[j] + gg.x[j] * gg.x[j];
                        x.x[j] = x.x[j] + (-U.lr) * gg.x[j] / (sqrtf(a.x[j]) + 1e-10f);
                    }
                    vstore(a, acc + row * D, (int)D, lane);
                }
                vstore(x, w + row * D, (int)D, lane);
                Vec z;
                vzero(z);
                vstore(z, gr + row * D, (int)D, lane);
                if (lane == 0) fl[row] = 0;
            }
            if (tid < threads) {   // the step consumed bs positives x dpp draws (Base.cpp:200-207 split)
                const int64_t per = bs % threads == 0 ? bs / threads : bs / threads + 1;
                int64_t len = bs - tid * per;
                len = len < 0 ? 0 : (len > per ? per : len);
                s_states[tid] = lcg_jump(s_states[tid], (uint64_t)(len * dpp));
            }
            if (tid == 0) epoch_loss += s_loss * P.inv_count + U.margin;
        }
        if (tid == 0 && U.losses) {
            U.losses[epoch] = epoch_loss;
        }
        epoch_loss = 0.f;
    }
    phase_barrier();
    if (tid < threads) U.states[tid] = s_states[tid];
}

}  // namespace dev

hipError_t launch_universes(const UniverseDev *d_us, int64_t n, const Shape &s, int model, int p_norm, int norm_flag,
                            int opt, int64_t neg, int bern, int filter, int64_t list_cap, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const dim3 grid((unsigned)n), block(256);
    const size_t lds = (size_t)list_cap * sizeof(int32_t);
#define PT_UNI(G_, V_, K_)                                                                                    \
    if (s.G == G_ && s.VEC == V_ && s.KCH == K_) {                                                          \
        if (model == 0)                                                                                       \
            hipLaunchKernelGGL((dev::k_universes<0, G_, V_, K_>), grid, block, lds, st, d_us, p_norm,        \
                               norm_flag, opt, neg, bern, filter);                                            \
        else                                                                                                  \
            hipLaunchKernelGGL((dev::k_universes<1, G_, V_, K_>), grid, block, lds, st, d_us, p_norm,        \
                               norm_flag, opt, neg, bern, filter);                                            \
        return hipGetLastError();                                                                           \
    }
    PT_SHAPES(PT_UNI)
#undef PT_UNI
    return hipErrorInvalidValue;
}

}  // namespace pt
