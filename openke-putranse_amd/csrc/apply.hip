// HIP kernels of the optimizer apply pass (sparse SGD / Adagrad rows) for gfx950.
//
// Layout and mapping
//  * Tables are row-major fp32 [rows][dim]. A "lane group" of G lanes (G | 64, a power of two) owns one
//    row-sized vector: lane l holds chunks c = k*G + l (k < KCH) of VEC consecutive floats, so a row is
//    read with fully coalesced 16-B (VEC=4) or 4-B (VEC=1) accesses and every reduction is a shuffle
//    butterfly inside the group. One positive triple and all its negatives belong to one group.
//  * This is gather/axpy work (no dense contraction): the roofline is HBM / Infinity-Cache bandwidth
//    and the memory-side float-atomic rate, not MFMA.
//
// Semantics (all cited in DESIGN.md): sampler = Base.cpp:185-310 + Corrupt.h:9-105 + Random.h:18-29;
// forward = TransE.py:46-74 / TransH.py:52-93; loss = MarginLoss.py:24-28 via NegativeSampling.py:13-31;
// backward = torch autograd of those ops (normalize Jacobian, sign / v/||v|| norm derivatives, maximum
// tie -> half); update = torch.optim.SGD / Adagrad (eps 1e-10) as built in Trainer.py:62-88, applied
// only to rows with a nonzero gradient (identical to the dense update).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "tuning.h"
#include "device.h"
#include "graph.h"
#include "kernels.h"
#include "rng.h"

namespace pt {
namespace dev {
using pt::CsrWork;

// Sparse apply: for every touched row finish the gradient (normalize Jacobian of the pre-step row
// when that table's gradient is in normalized space) and run SGD / Adagrad; then clear the row.
struct ApplyTable {
    float *w, *acc, *grad;
    int *flag;
    int64_t rows;
    int jacobian;
    const int *start;       // CSR of extra contribution rows (NULL: none): rows start[r] .. start[r+1]-1
    const float *contrib;   // [n][dim]
};
struct ApplyParams {
    ApplyTable t[3];
    int ntab;
    int64_t dim;
    int opt;
    float lr;
    // sampler advance + loss (done by block 0)
    uint64_t *states;
    int64_t threads, bs, dpp;
    float *loss;
    const float *lpart;   // [bs] per-positive loss partials of the step
    float margin, inv_count;
    int dbg;   // timing experiments only (PT_STEP_DBG bit 3: contribution rows read from a 4096-row hot window)
    int loss_assign;
    // slot-scale mode (CsrWork::slot_scale): the step's slot records and positive base rows, the model's p and
    // norm_flag (k_apply_buf<..., true>)
    const int2 *srec;
    const float *bases;
    int p_norm, norm_flag;
};

// block 0, first wave: advance the sampler streams and reduce the step's loss partials in a fixed
// order: loss += inv_count * sum(lpart) + margin (MarginLoss.py:24-28)
__device__ __forceinline__ void apply_block0(const ApplyParams &A) {
    const int lane = (int)threadIdx.x;
    if (A.states) advance_states(A.states, A.threads, A.bs, A.dpp, lane);
    if (A.loss && A.lpart) {
        float s = 0.f;
        for (int64_t i0 = lane; i0 < A.bs; i0 += 64 * 8) {   // 8 independent loads in flight per lane
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = i0 + u * 64 < A.bs ? A.lpart[i0 + u * 64] : 0.f;
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        s = gsum<64>(s);
        if (lane == 0) {
            const float l = s * A.inv_count + A.margin;
            if (A.loss_assign) *A.loss = l; else *A.loss += l;
        }
    }
}

template <int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_apply(ApplyParams A) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    const int lane = threadIdx.x % G;
    int64_t row = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    if (blockIdx.x == 0 && threadIdx.x < 64) apply_block0(A);
    int ti = 0;
    while (ti < A.ntab && row >= A.t[ti].rows) {
        row -= A.t[ti].rows;
        ++ti;
    }
    if (ti >= A.ntab) return;
    const ApplyTable &T = A.t[ti];
    const int flagged = T.flag[row];
    int c0 = 0, c1 = 0;
    if (T.start) {
        c0 = T.start[row];
        c1 = T.start[row + 1];
    }
    if (!flagged && c0 == c1) return;
    const int D = (int)A.dim;
    Vec x, gsum_, g;
    vload(x, T.w + row * D, D, lane);
    if (flagged) vload(gsum_, T.grad + row * D, D, lane); else vzero(gsum_);
    // contributions of this step's corrupted-entity slots (counting-sort order)
    int j = c0;
    for (; j + 4 <= c1; j += 4) {
        Vec c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) vload(c[u], T.contrib + (int64_t)(j + u) * D, D, lane);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) gsum_.x[i] += c[u].x[i];
    }
    for (; j < c1; ++j) {
        Vec c;
        vload(c, T.contrib + (int64_t)j * D, D, lane);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) gsum_.x[i] += c.x[i];
    }
    if (T.jacobian) {
        const float n = sqrtf(vdot(x, x));
        vnormalize_bwd(x, n, gsum_, g);
    } else {
        g = gsum_;
    }
    if (A.opt == 0) {
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) x.x[i] = x.x[i] + (-A.lr) * g.x[i];
    } else {
        Vec a;
        vload(a, T.acc + row * D, D, lane);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            a.x[i] = a.x[i] + g.x[i] * g.x[i];
            x.x[i] = x.x[i] + (-A.lr) * g.x[i] / (sqrtf(a.x[i]) + 1e-10f);
        }
        vstore(a, T.acc + row * D, D, lane);
    }
    vstore(x, T.w + row * D, D, lane);
    if (flagged) {
        Vec z;
        vzero(z);
        vstore(z, T.grad + row * D, D, lane);
        if (lane == 0) T.flag[row] = 0;
    }
}

// Apply pass with float4 rows and raw-buffer access (D % 4 == 0, offsets within 31 bits): one lane
// group per table row. The row (and its Adagrad state) load is issued before the flag / bucket range
// loads return; a bucket's contribution rows stream NC at a time with out-of-range offsets past its
// end (the hardware returns zeros, so the adds need no branches), summed in bucket order after the
// row's own gradient row.
template <int G, int VEC, int KCH, int NC, int RPW, bool SC = false>
__global__ __launch_bounds__(256) void k_apply_buf(ApplyParams A) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    const int lane = threadIdx.x % G;
    const int64_t gi = uni<G>((int32_t)(blockIdx.x * GPB + threadIdx.x / G));   // scalar at G = 64
    if (blockIdx.x == 0 && threadIdx.x < 64) apply_block0(A);
    const int D = (int)A.dim;
    const uint32_t rowb = (uint32_t)D * 4u;
    // RPW consecutive rows per group, every load of all of them in flight together
    int ti[RPW], flag[RPW], c0[RPW], c1[RPW];
    int64_t row[RPW];
    bool live[RPW];
    Vec x[RPW], g[RPW], a[RPW];
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        int64_t r = gi * RPW + u;
        int t = 0;
        while (t < A.ntab && r >= A.t[t].rows) {
            r -= A.t[t].rows;
            ++t;
        }
        ti[u] = t;
        row[u] = r;
        live[u] = t < A.ntab;
        flag[u] = 0;
        c0[u] = c1[u] = 0;
    }
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        if (!live[u]) continue;
        const ApplyTable &T = A.t[ti[u]];
        const uint32_t tb = (uint32_t)T.rows * rowb;
        bload(x[u], make_rsrc(T.w, tb), (uint32_t)row[u] * rowb, D, lane);
        if (A.opt != 0) bload(a[u], make_rsrc(T.acc, tb), (uint32_t)row[u] * rowb, D, lane);
        flag[u] = T.flag[row[u]];
        if (T.start) {
            c0[u] = T.start[row[u]];
            c1[u] = T.start[row[u] + 1];
        }
    }
    int len = 0;
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        if (!live[u]) continue;
        const ApplyTable &T = A.t[ti[u]];
        bload(g[u], make_rsrc(T.grad, (uint32_t)T.rows * rowb), flag[u] ? (uint32_t)row[u] * rowb : kOob, D, lane);
        len = c1[u] - c0[u] > len ? c1[u] - c0[u] : len;
    }
    if constexpr (SC) {
#pragma clang fp contract(off)   // (k v and the sum stay two roundings, as the stored row and its add were)
        // slot-scale mode (CsrWork::slot_scale): each slot's row re-formed from its record and its positive's
        // normalized rows with the step kernel's own operations - e-hat = normalize(x) (fast form), v = b-hat - e-hat
        // (a corrupted tail) or (e-hat + r-hat) - t-hat (a corrupted head), then k v (p = 2) or k sign(v) (p = 1)
        // - and summed in bucket order: the bits the stored contribution rows held
        const auto b_rs = make_rsrc(A.bases, 0x7fffffffu);
#pragma unroll
        for (int u = 0; u < RPW; ++u) {
            if (!live[u] || ti[u] != 0 || c0[u] == c1[u]) continue;
            Vec eh;
            if (A.norm_flag) vnormalize<true>(x[u], eh); else eh = x[u];
            for (int j = c0[u]; j < c1[u]; j += NC) {
                int2 rc[NC];
#pragma unroll
                for (int q = 0; q < NC; ++q) {
                    const int2 r = j + q < c1[u] ? A.srec[j + q] : make_int2(0, 0);
                    rc[q] = make_int2(uni<G>(r.x), uni<G>(r.y));
                }
                Vec ra[NC], rb[NC];
#pragma unroll
                for (int q = 0; q < NC; ++q) {
                    const bool ok = j + q < c1[u];
                    const uint32_t pb = (uint32_t)(rc[q].x >> 1) * 3u;
                    const bool tail = rc[q].x & 1;
                    bload(ra[q], b_rs, ok ? (tail ? pb : pb + 1u) * rowb : kOob, D, lane);
                    bload(rb[q], b_rs, ok && !tail ? (pb + 2u) * rowb : kOob, D, lane);
                }
#pragma unroll
                for (int q = 0; q < NC; ++q) {
                    if (j + q >= c1[u]) break;
                    const bool tail = rc[q].x & 1;
                    const float kk = __int_as_float(rc[q].y);
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) {
                        const float vk = tail ? ra[q].x[i] - eh.x[i] : (eh.x[i] + ra[q].x[i]) - rb[q].x[i];
                        const float gs = A.p_norm == 1 ? (vk > 0.f ? kk : (vk < 0.f ? -kk : 0.f)) : vk * kk;
                        g[u].x[i] += gs;
                    }
                }
            }
        }
    } else {
    // contribution rows (entity table only): the rows' buckets streamed side by side, NC per row at a
    // time, out-of-range past each bucket's end (zeros), summed in bucket order
    const auto c_rs = make_rsrc(A.t[0].contrib, 0x7fffffffu);
    for (int j = 0; j < len; j += NC) {
        Vec c[RPW][NC];
#pragma unroll
        for (int u = 0; u < RPW; ++u)
#pragma unroll
            for (int q = 0; q < NC; ++q)
                bload(c[u][q], c_rs,
                      c0[u] + j + q < c1[u] ? (uint32_t)(PT_ABLATE(A.dbg, 8) ? (c0[u] + j + q) & 4095 : c0[u] + j + q) * rowb
                                            : kOob,
                      D, lane);
#pragma unroll
        for (int u = 0; u < RPW; ++u)
#pragma unroll
            for (int q = 0; q < NC; ++q)
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) g[u].x[i] += c[u][q].x[i];
    }
    }
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        if (!live[u] || (!flag[u] && c0[u] == c1[u])) continue;   // untouched row: unchanged
        const ApplyTable &T = A.t[ti[u]];
        const uint32_t tb = (uint32_t)T.rows * rowb;
        Vec gg;
        if (T.jacobian) {
            const float n = sqrtf(vdot(x[u], x[u]));
            vnormalize_bwd(x[u], n, g[u], gg);
        } else {
            gg = g[u];
        }
        if (A.opt == 0) {
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) x[u].x[i] = x[u].x[i] + (-A.lr) * gg.x[i];
        } else {
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) {
                a[u].x[i] = a[u].x[i] + gg.x[i] * gg.x[i];
                x[u].x[i] = x[u].x[i] + (-A.lr) * gg.x[i] / (sqrtf(a[u].x[i]) + 1e-10f);
            }
            bstore(a[u], make_rsrc(T.acc, tb), (uint32_t)row[u] * rowb, D, lane);
        }
        bstore(x[u], make_rsrc(T.w, tb), (uint32_t)row[u] * rowb, D, lane);
        if (flag[u]) {
            Vec z;
            vzero(z);
            bstore(z, make_rsrc(T.grad, tb), (uint32_t)row[u] * rowb, D, lane);
            if (lane == 0) T.flag[row[u]] = 0;
        }
    }
}

// Apply pass, RPW consecutive rows per lane group with all their loads in flight together (the
// one-row-per-group form is a chain of two dependent memory round trips per row). Consecutive entity
// rows own consecutive counting-sort contribution ranges, so a group streams ONE contiguous range
// [start[r0], start[r0 + RPW]) and adds each contribution to its row.
template <int G, int VEC, int KCH, int RPW>
__global__ __launch_bounds__(256) void k_apply_rows(ApplyParams A) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    const int lane = threadIdx.x % G;
    const int64_t gi = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    if (blockIdx.x == 0 && threadIdx.x < 64) apply_block0(A);
    const int D = (int)A.dim;
    int ti[RPW];
    int64_t row[RPW];
    int flag[RPW], c0[RPW], c1[RPW];
    bool live[RPW];
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        int64_t r = gi * RPW + u;
        int t = 0;
        while (t < A.ntab && r >= A.t[t].rows) {
            r -= A.t[t].rows;
            ++t;
        }
        ti[u] = t;
        row[u] = r;
        flag[u] = 0;
        c0[u] = c1[u] = 0;
        if (t < A.ntab) {
            flag[u] = A.t[t].flag[r];
            if (A.t[t].start) {
                c0[u] = A.t[t].start[r];
                c1[u] = A.t[t].start[r + 1];
            }
        }
        live[u] = t < A.ntab && (flag[u] || c0[u] != c1[u]);
    }
    Vec x[RPW], g[RPW], a[RPW];
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        if (!live[u]) continue;
        const ApplyTable &T = A.t[ti[u]];
        vload(x[u], T.w + row[u] * D, D, lane);
        if (flag[u]) vload(g[u], T.grad + row[u] * D, D, lane); else vzero(g[u]);
        if (A.opt != 0) vload(a[u], T.acc + row[u] * D, D, lane);
    }
    // the group's contribution range (entity table rows only carry contributions)
    int cs = 0, ce = 0;
    bool any = false;
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        if (c0[u] == c1[u]) continue;
        if (!any) cs = c0[u];
        ce = c1[u];
        any = true;
    }
    if (any) {
        const float *contrib = A.t[0].contrib;
        for (int j = cs; j < ce; j += 4) {
            Vec c[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (j + q < ce) vload(c[q], contrib + (int64_t)(j + q) * D, D, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (j + q >= ce) break;
#pragma unroll
                for (int u = 0; u < RPW; ++u) {
                    if (j + q >= c0[u] && j + q < c1[u]) {
#pragma unroll
                        for (int i = 0; i < Vec::N; ++i) g[u].x[i] += c[q].x[i];
                    }
                }
            }
        }
    }
#pragma unroll
    for (int u = 0; u < RPW; ++u) {
        if (!live[u]) continue;
        const ApplyTable &T = A.t[ti[u]];
        Vec gg;
        if (T.jacobian) {
            const float n = sqrtf(vdot(x[u], x[u]));
            vnormalize_bwd(x[u], n, g[u], gg);
        } else {
            gg = g[u];
        }
        if (A.opt == 0) {
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) x[u].x[i] = x[u].x[i] + (-A.lr) * gg.x[i];
        } else {
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) {
                a[u].x[i] = a[u].x[i] + gg.x[i] * gg.x[i];
                x[u].x[i] = x[u].x[i] + (-A.lr) * gg.x[i] / (sqrtf(a[u].x[i]) + 1e-10f);
            }
            vstore(a[u], T.acc + row[u] * D, D, lane);
        }
        vstore(x[u], T.w + row[u] * D, D, lane);
        if (flag[u]) {
            Vec z;
            vzero(z);
            vstore(z, T.grad + row[u] * D, D, lane);
            if (lane == 0) T.flag[row[u]] = 0;
        }
    }
}

}  // namespace dev

// ==================================================================== host launchers ===========
hipError_t launch_apply(const StepParams &P, const StepWorkspace &W, uint64_t *states, int64_t threads, int64_t bs,
                        int64_t dpp, float *loss, hipStream_t st, const CsrWork *csr) {
    const Shape s = pick_shape(P.dim);
    dev::ApplyParams A{};
    A.ntab = 0;
    const int ent_j = P.model == 0 && P.norm_flag;
    A.t[A.ntab++] = dev::ApplyTable{P.ent, P.ent_acc, W.gent, W.fent, P.ent_total, ent_j,
                                    csr ? csr->start : nullptr, csr ? csr->contrib : nullptr};
    A.t[A.ntab++] = dev::ApplyTable{P.rel, P.rel_acc, W.grel, W.frel, P.rel_total, P.norm_flag, nullptr, nullptr};
    if (P.model == 1)
        A.t[A.ntab++] = dev::ApplyTable{P.normv, P.norm_acc, W.gnorm, W.fnorm, P.rel_total, 1, nullptr, nullptr};
    A.dim = P.dim;
    A.opt = P.opt;
    A.lr = P.lr;
    A.states = states;
    A.threads = threads;
    A.bs = bs;
    A.dpp = dpp;
    A.loss = loss;
    A.lpart = W.lpart;
    A.margin = P.margin;
    A.inv_count = P.inv_count;
    A.dbg = P.dbg;
    A.loss_assign = P.loss_assign;
    const bool sc = csr && csr->slot_scale;
    A.srec = sc ? csr->srec : nullptr;
    A.bases = sc ? csr->bases : nullptr;
    A.p_norm = P.p_norm;
    A.norm_flag = P.norm_flag;
    int64_t rows = 0;
    for (int i = 0; i < A.ntab; ++i) rows += A.t[i].rows;
    // float4 rows through raw buffers (PT_APPLY_OLD=1 keeps the kernels below)
    static const bool old_apply = [] {
        const char *v = pt_tuning_env("PT_APPLY_OLD");
        return v && atoi(v) != 0;
    }();
    int64_t con_rows = 0;
    if (csr) con_rows = P.batch_size * P.neg;
    const bool fits31 = (P.ent_total + P.rel_total + con_rows) * P.dim * 4 < (int64_t(1) << 31);
    if (P.dim % 4 == 0 && fits31 && !old_apply) {
        const int64_t chunks = P.dim / 4;
        int G = 2;
        while (G < chunks && G < 64) G <<= 1;
        const int KCH = (int)((chunks + G - 1) / G);
        // contribution rows in flight per lane group: 8 for one-chunk float4 rows (C2: the bucket of a row
        // - Poisson, mean 3.6 at C2 - mostly in one round trip; measured 12.0 vs 12.6 us), else 4
        int nc = G == 64 && KCH == 1 ? 8 : 4, rpw = 1;
        if (const char *v = pt_tuning_env("PT_APPLY_NC")) nc = atoi(v);
        if (const char *v = pt_tuning_env("PT_APPLY_RPW")) rpw = atoi(v);
        const int64_t gpb4 = 256 / G;
        const int64_t groups = (rows + rpw - 1) / rpw;
        const dim3 grid((unsigned)((groups + gpb4 - 1) / gpb4)), block(256);
#define PT_APPLYB(G_, K_, N_, R_)                                                              \
        if (G == G_ && KCH == K_ && nc == N_ && rpw == R_) {                                  \
            if (sc)                                                                             \
                hipLaunchKernelGGL((dev::k_apply_buf<G_, 4, K_, N_, R_, true>), grid, block, 0, st, A); \
            else                                                                                \
                hipLaunchKernelGGL((dev::k_apply_buf<G_, 4, K_, N_, R_>), grid, block, 0, st, A); \
            return hipGetLastError();                                                         \
        }
        PT_APPLYB(2, 1, 4, 1) PT_APPLYB(4, 1, 4, 1) PT_APPLYB(8, 1, 4, 1) PT_APPLYB(16, 1, 4, 1)
        PT_APPLYB(32, 1, 4, 1) PT_APPLYB(64, 1, 4, 1) PT_APPLYB(64, 2, 4, 1) PT_APPLYB(64, 3, 4, 1)
        PT_APPLYB(64, 4, 4, 1) PT_APPLYB(64, 1, 2, 1) PT_APPLYB(64, 1, 4, 2) PT_APPLYB(64, 1, 2, 2) PT_APPLYB(64, 1, 8, 1)
        PT_APPLYB(64, 1, 2, 4) PT_APPLYB(64, 1, 1, 4)
#undef PT_APPLYB
    }
    if (sc) return hipErrorInvalidValue;   // slot records are read only by k_apply_buf
    const int64_t gpb = 256 / s.G;
    // PT_APPLY_RPW=2|4: several rows per lane group with one contribution stream (measured slower on
    // C2: 20.4 / 22.0 us vs 16.8 us for one row per group, which stays the default)
    const char *rpw_env = pt_tuning_env("PT_APPLY_RPW");
    const int rpw = rpw_env ? atoi(rpw_env) : 1;
    if (rpw == 4 || rpw == 2) {
        const int64_t groups = (rows + rpw - 1) / rpw;
        const dim3 grid((unsigned)((groups + gpb - 1) / gpb)), block(256);
#define PT_APPLY4(G_, V_, K_)                                                                 \
        if (s.G == G_ && s.VEC == V_ && s.KCH == K_) {                                      \
            if (rpw == 4)                                                                   \
                hipLaunchKernelGGL((dev::k_apply_rows<G_, V_, K_, 4>), grid, block, 0, st, A); \
            else                                                                            \
                hipLaunchKernelGGL((dev::k_apply_rows<G_, V_, K_, 2>), grid, block, 0, st, A); \
            return hipGetLastError();                                                       \
        }
        PT_SHAPES(PT_APPLY4)
#undef PT_APPLY4
    }
    const dim3 grid((unsigned)((rows + gpb - 1) / gpb)), block(256);
#define PT_APPLY(G_, V_, K_)                                                                  \
    if (s.G == G_ && s.VEC == V_ && s.KCH == K_) {                                          \
        hipLaunchKernelGGL((dev::k_apply<G_, V_, K_>), grid, block, 0, st, A);              \
        return hipGetLastError();                                                           \
    }
    PT_SHAPES(PT_APPLY)
#undef PT_APPLY
    return hipErrorInvalidValue;
}

}  // namespace pt
