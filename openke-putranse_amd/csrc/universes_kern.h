// Persistent multi-universe trainer (PuTransE / PuTransH, BASELINE configs C3-C5): device code, included by
// universes.hip (host side, LDS plan 0) and universes_p1.hip / universes_p2.hip (plans 1 and 2, compiled apart).
//
// The reference trains its universes one after another, each with Trainer.run over
// epochs x nbatches tiny minibatches (Parallel_Universe_Config.py:228-258, Trainer.py:90-104); a
// universe step is ~25-100 positives, far too small for a launch per step. Here ONE workgroup owns
// ONE universe for its whole training run: every epoch and minibatch is a loop iteration inside the
// kernel, with two workgroup barriers per step that give the reference's minibatch-synchronous
// semantics (every gradient of a step sees the pre-step tables):
//
//   sample   every `pchunk` steps the next pchunk batches (TrainDataLoader.sampling() calls) are drawn
//            at once into LDS, lane-parallel (stream jumps, rng.h);
//   phase A  each lane group takes positives b = grp, grp + GPB, ... of the step and runs group_step
//            (forward, MarginLoss, backward). Gradient rows leave it through the sink:
//              entity rows  -> written with plain stores to a per-universe contribution slot and
//                              linked into the row's LDS list (no float atomics: 512 universes x
//                              ~40 K row-element atomics per step saturate the L2 atomic units);
//              relation / norm_vector rows -> LDS float atomics into LDS gradient rows (a universe
//                              has few relations, and every positive of a step hits its relation);
//            the first touch of a row appends it to an LDS work list;
//   phase B  lane groups walk the work list, RB rows at a time: sum the row's contributions, normalize
//            Jacobian of the pre-step row where the gradient is in normalized space, Adagrad (or SGD)
//            update, reset the row's LDS state.
//
// Whatever does not fit the LDS budget falls back to global memory (atomic gradient rows, flag arrays,
// per-step sampling). Universes are independent, so thousands run concurrently (one per workgroup,
// several per CU); universes of different row shapes run as separate launches on separate streams.
#pragma once
#include <hip/hip_runtime.h>

// Tuning build only: s_memtime stamps of one step's rounds (lane group 0) into the profiling record
#ifdef PT_TUNING
#define PT_USTAMP(ptr, i) do { if ((ptr) && lane == 0) (ptr)[i] = clock64(); } while (0)
#else
#define PT_USTAMP(ptr, i) do { } while (0)
#endif

#include <cstdint>
#include <cstdlib>

#include "tuning.h"
#include "device.h"
#include "kernels.h"
#include "universes.h"

namespace pt {
namespace dev {

// release / acquire at agent scope around the workgroup barrier: stores of one phase are visible to
// loads of the next phase from any wave (L1 invalidated), independent of L1 write policy
// (needed while gradient rows are float atomics performed at L2: a later plain load must not hit a
// stale L1 line). Without global atomics in the step (contribution lists + LDS relation rows + LDS
// flags) every cross-wave exchange is plain stores / loads or LDS within the workgroup, which the
// workgroup barrier alone orders (all waves of a workgroup share the CU's L1).
__device__ __forceinline__ void phase_barrier(bool agent) {
    if (agent) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    } else {
        __syncthreads();
    }
}

// Hardware sqrt / reciprocal (1 ulp, v_sqrt_f32 / v_rcp_f32), as in the C2 training step, for the row
// shapes of at most 8 floats per lane: a correctly rounded division or square root is ~10 VALU
// instructions in a kernel bound by instruction issue. The 16-float class (TransE rows over 512 floats since
// r04; C4's D = 200 before) keeps the IEEE forms: with the hardware forms its register allocation slowed its
// phase A by 25% (r03, C4 105 -> 120 ms). (A 1-ulp difference amplified by a cancelling gradient sum, 5.3e-6
// on one C4 component in r03, is within the forward-error bound the parity tests use since r04.) The
// reference-order kernel (ordered.hip) keeps IEEE forms throughout.
constexpr bool kUF = true;
// PT_UNI_FAST_WIDE=0 (measurement builds): the wide rows (lane groups of 32 / 64 lanes: C4's D = 200) take the IEEE
// forms too
#ifndef PT_UNI_FAST_WIDE
#define PT_UNI_FAST_WIDE 1
#endif
// PT_UNI_LIST_BATCH (measurement builds): the contribution rows a plan-2 relation row's phase-B walk keeps in flight
#ifndef PT_UNI_LIST_BATCH
#define PT_UNI_LIST_BATCH 4
#endif
constexpr bool uni_fast(int G, int floats) { return kUF && floats <= 8 && (PT_UNI_FAST_WIDE || G < 32); }

// backward of F.normalize (vnormalize_bwd) without a branch on the norm: the rows of a wave's lane groups
// take the (g - x (x.g)/n^2) / n form or the clamp's g / eps form by selects, not by divergent paths
template <bool FAST, int G, int VEC, int KCH>
__device__ __forceinline__ void unormalize_bwd(const V<G, VEC, KCH> &x, float n, const V<G, VEC, KCH> &g,
                                               V<G, VEC, KCH> &out) {
    const bool big = n > kEps;
    const float inv = big ? frcp<FAST>(n) : 1.0f / kEps;
    const float c = big ? vdot(g, x) * (inv * inv) : 0.f;
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) out.x[i] = (g.x[i] - x.x[i] * c) * inv;
}

// Rows of up to 128 floats (16 lanes or fewer) take KCH = ceil(chunks / G) chunks per lane instead of the next
// power of two: e.g. D = 69 on 16 lanes holds 5 floats per lane, not 8 (C3 48.3 -> 43.3 ms, the longest
// universe's phase A 21.1k -> 19.2k cycles/step); G = 2 rows and longer rows keep power-of-two chunk counts
// (2-lane groups: any KCH <= p is already exact; G = 32 / 64: fewer shapes per class kernel)
constexpr bool exact_kch_shape(int G, int VEC) { return G >= (VEC == 4 ? 2 : 4) && G <= (VEC == 4 ? 8 : 16); }

// Row access of the universe kernels. HBM-typed (global_load / global_store: they count in vmcnt only, so a
// wait for an LDS read - the batch, the contribution lists - never waits for row traffic in flight, as a flat
// access would) and branch-free: every chunk of an exact shape but its last is full for every dim the shape
// takes (pick_universe_shape: D in ((KCH - 1) G VEC, KCH G VEC]), so those chunks load unconditionally; the
// last (and every chunk of the power-of-two shapes) loads from a clamped in-row address and selects zero past
// the row's end, instead of an exec-masked branch per chunk. Stores skip only lanes past the end.
// Used by the classes of at most 8 floats per lane (same-box A/B, r04: C5 37.2 -> 36.6 ms); the 16-float
// class keeps the generic (flat, masked) vload / vstore of device.h (C4 105.6 ms flat vs 121 ms typed: its
// longer branch-free chunk sequences raised its register allocation). PT_UNI_GLOBAL (measurement builds):
// 0 = flat everywhere, 1 = typed everywhere, 2 = typed up to 8 floats per lane (default).
#ifndef PT_UNI_GLOBAL
#define PT_UNI_GLOBAL 2
#endif
constexpr bool uni_global(int floats) { return PT_UNI_GLOBAL == 1 || (PT_UNI_GLOBAL == 2 && floats <= 8); }
template <int G, int VEC, int KCH>
constexpr int full_chunks() { return exact_kch_shape(G, VEC) ? KCH - 1 : 0; }

template <int G, int VEC, int KCH>
__device__ __forceinline__ void uload(V<G, VEC, KCH> &o, const float *row_, int D, int lane) {
    if constexpr (!uni_global(VEC * KCH)) {
        vload(o, row_, D, lane);
        return;
    }
    const gfloat *row = (const gfloat *)(const void *)row_;
    constexpr int F = full_chunks<G, VEC, KCH>();
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        const bool ok = k < F || c * VEC < D;
        const int cc = k < F ? c : (ok ? c : 0);   // chunk 0 is inside every row
        if constexpr (VEC == 4) {
            const f32x4 f = *reinterpret_cast<const gf32x4 *>(row + cc * 4);
            o.x[k * 4 + 0] = ok ? f.x : 0.f; o.x[k * 4 + 1] = ok ? f.y : 0.f;
            o.x[k * 4 + 2] = ok ? f.z : 0.f; o.x[k * 4 + 3] = ok ? f.w : 0.f;
        } else {
#pragma unroll
            for (int q = 0; q < VEC; ++q) {
                const float v = row[cc * VEC + q];
                o.x[k * VEC + q] = ok ? v : 0.f;
            }
        }
    }
}

template <int G, int VEC, int KCH>
__device__ __forceinline__ void ustore(const V<G, VEC, KCH> &o, float *row_, int D, int lane) {
    if constexpr (!uni_global(VEC * KCH)) {
        vstore(o, row_, D, lane);
        return;
    }
    gfloat *row = (gfloat *)(void *)row_;
    constexpr int F = full_chunks<G, VEC, KCH>();
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if (k < F || c * VEC < D) {
            if constexpr (VEC == 4) {
                const f32x4 f = {o.x[k * 4 + 0], o.x[k * 4 + 1], o.x[k * 4 + 2], o.x[k * 4 + 3]};
                *reinterpret_cast<gf32x4 *>(row + c * 4) = f;
            } else {
#pragma unroll
                for (int q = 0; q < VEC; ++q) row[c * VEC + q] = o.x[k * VEC + q];
            }
        }
    }
}

// Adds the contribution rows of an LDS-linked list (slot c, next[c], ...) to gs, in list order. BATCH > 1: the next
// BATCH slot ids are read down the LDS chain first and their rows loaded together - one load latency per BATCH rows
// instead of one per row (a relation row of a plan-2 universe - C4's 121 relations, C5's TransH rows - collects tens
// of contributions per step, walked one dependent load at a time before round 6). load(Vec &, slot).
template <int BATCH, int G, int VEC, int KCH, typename Load>
__device__ __forceinline__ void list_sum(V<G, VEC, KCH> &gs, int32_t c, const int32_t *next, Load load) {
    using Vec = V<G, VEC, KCH>;
    if constexpr (BATCH <= 1) {
        for (; c >= 0; c = next[c]) {
            Vec y;
            load(y, c);
#pragma unroll
            for (int j = 0; j < Vec::N; ++j) gs.x[j] += y.x[j];
        }
    } else {
        while (c >= 0) {
            int32_t cc[BATCH];
            cc[0] = c;
#pragma unroll
            for (int k = 1; k < BATCH; ++k) cc[k] = cc[k - 1] >= 0 ? next[cc[k - 1]] : -1;
            Vec y[BATCH];
#pragma unroll
            for (int k = 0; k < BATCH; ++k)
                if (cc[k] >= 0) load(y[k], cc[k]);
#pragma unroll
            for (int k = 0; k < BATCH; ++k)
                if (cc[k] >= 0) {
#pragma unroll
                    for (int j = 0; j < Vec::N; ++j) gs.x[j] += y[k].x[j];
                }
            c = cc[BATCH - 1] >= 0 ? next[cc[BATCH - 1]] : -1;
        }
    }
}

// Gradient sink of one universe.
//   contrib != null: entity rows go to contribution slots (plain stores) linked per row in LDS
//   (head[row] -> c -> next[c] -> ... -> -1); otherwise float atomics into gent.
//   grel / gnorm point to LDS gradient rows or to global ones (float atomics either way).
template <int PLAN>
struct UniverseSink {
    float *gent, *grel, *gnorm;
    int32_t *fent, *frel, *fnorm;
    int32_t *list;
    int *count;
    float *contrib;      // [ccap][D] (global) or null: entity rows as contribution lists
    int32_t *head;       // [E + 2R] LDS list heads (entity rows, then relation rows, then norm_vector rows)
    int32_t *next;       // [ccap] LDS
    int *ccount;         // LDS counter of contribution slots
    int E, R;
    bool rel_list;       // relation / norm_vector rows as contribution lists too
    // next contribution slot of the lane group's current positive: positive b owns the static slots
    // [b * per_pos, (b + 1) * per_pos), per_pos = neg + 2 (+2 with relation lists) >= its links
    mutable int slot = 0;
    uint64_t *trace = nullptr;   // tuning build: phase stamps of this positive (null: none)
    __device__ __forceinline__ void touch(int32_t *flag, int row, int table) const {
        if (atomicExch(flag + row, 1) == 0) list[atomicAdd(count, 1)] = (int32_t)(row << 2) | table;
    }
    // plain store of the row gradient into a fresh contribution slot, linked into the row's list
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void link(int32_t *h, int row, int table, const V<G, VEC, KCH> &g, int D,
                                         int lane) const {
        const int c = slot++;   // group-uniform: every lane of the group makes the same calls
        ustore(g, contrib + c * D, D, lane);
        if (lane == 0) {
            const int32_t prev = atomicExch(h + row, c);
            next[c] = prev;
            if (prev < 0) list[atomicAdd(count, 1)] = (int32_t)(row << 2) | table;
        }
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void ent(int row, const V<G, VEC, KCH> &g, int D, int lane) const {
        if (PLAN != 0 || contrib) {
            link(head, row, 0, g, D, lane);
        } else {
            vatomic(g, gent + row * D, D, lane);
            if (lane == 0) touch(fent, row, 0);
        }
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void rel(int row, const V<G, VEC, KCH> &g, int D, int lane) const {
        if (PLAN == 2 || (PLAN == 0 && rel_list)) {
            link(head + E, row, 1, g, D, lane);
        } else {
            vatomic(g, grel + row * D, D, lane);
            if (lane == 0) touch(frel, row, 1);
        }
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void norm(int row, const V<G, VEC, KCH> &g, int D, int lane) const {
        if (PLAN == 2 || (PLAN == 0 && rel_list)) {
            link(head + E + R, row, 2, g, D, lane);
        } else {
            vatomic(g, gnorm + row * D, D, lane);
            if (lane == 0) touch(fnorm, row, 2);
        }
    }
};

// TransE step of NP positives (one lane group, their chains interleaved; measured with NP = 2 for the rows of
// at most 8 floats per lane: C3 49.0 -> 55.0 ms, the class kernel then spills 98 VGPRs; NP = 1 is used) whose negatives
// each replace ONE side with entity e (the sampler's structure, Base.cpp:217-232): the same forward /
// MarginLoss / backward as group_step with a smaller live set (normalized rows kept in place, no
// per-negative row-role bookkeeping). get_neg(q, k, &e, &tail_side). Gradients in normalized space, like
// group_step for TransE; a corrupted row equal to a positive row is simply a separate contribution.
// Positive q's gradient rows go to sink sk[q] (its own contribution slots). Returns the summed losses.
// Row of a universe table for transe_step: SC1 (a team universe, universes_team.h) loads it past the CU's L1 with
// sc1 buffer loads (rows another team member updated), else uload.
template <bool SC1, int G, int VEC, int KCH>
__device__ __forceinline__ void trow(V<G, VEC, KCH> &o, const float *table, int64_t rows, int row, int D, int lane) {
    if constexpr (SC1)
        bload<G, VEC, KCH, 16>(o, make_rsrc(table, (uint32_t)(rows * D * 4)), (uint32_t)(row * D * 4), D, lane);
    else
        uload(o, table + row * D, D, lane);
}

// ALWAYS (team universes): every row of the positive goes to its sink, a zero row for an inactive pair, so each
// positive fills its static contribution slots (neg negatives, relation, head, tail) whatever its margin decisions.
template <int NP, int G, int VEC, int KCH, bool PF = false, bool ALWAYS = false, bool SC1 = false, typename Sink,
          typename NegFn>
__device__ __forceinline__ float transe_step(const StepParams &P, const int (&hp)[NP], const int (&rp)[NP],
                                             const int (&tp)[NP], int neg, NegFn get_neg, const Sink (&sk)[NP],
                                             int lane) {
    using Vec = V<G, VEC, KCH>;
    constexpr bool kFm = uni_fast(G, VEC * KCH);   // hardware sqrt / rcp (see kUF)
    const int D = (int)P.dim;
    const int p = P.p_norm;
    const bool nf = P.norm_flag != 0;
    PT_USTAMP(sk[0].trace, 0);
    Vec hh[NP], th[NP], rh[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        trow<SC1>(hh[q], P.ent, P.ent_total, hp[q], D, lane);
        trow<SC1>(th[q], P.ent, P.ent_total, tp[q], D, lane);
        trow<SC1>(rh[q], P.rel, P.rel_total, rp[q], D, lane);
    }
    // long wide rows (16 floats per lane over >= 16 lanes: TransE rows over 512 floats since r04): the first
    // negative's row loads with the positive's, the rest one at a time in the loop (measured r02 on C4's then
    // 16-float rows, D = 200: 129 -> 108 ms; for
    // the short rows of C3 the extra live row costs more than the round trip it hides, 66 -> 74 ms)
    // (for every shape: C3 / C4 / C5 unchanged, r03; measured r04 and removed: also prefetching for the rows
    // of at most 6 floats per lane with the four rows' normalizations and the two score norms reduced
    // together (grouped DPP reductions) - C3 53.7 -> 55.5 ms, C5 (TransH counterpart) 36.6 -> 37.5 ms)
    constexpr bool kPrefetch = PF || (VEC * KCH >= 16 && G >= 16);   // PF: see universe_run
    int e[NP];
    bool tail_side[NP];
    Vec x[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        e[q] = 0;
        tail_side[q] = false;
        if (kPrefetch && neg > 0) {
            get_neg(q, 0, e[q], tail_side[q]);
            trow<SC1>(x[q], P.ent, P.ent_total, e[q], D, lane);
        }
    }
    float ps[NP], csum[NP], lsum[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        if (nf) {
            vnormalize<kFm>(hh[q], hh[q]);
            vnormalize<kFm>(rh[q], rh[q]);
            vnormalize<kFm>(th[q], th[q]);
        }
        Vec vpos;
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) vpos.x[i] = (hh[q].x[i] + rh[q].x[i]) - th[q].x[i];
        ps[q] = vpnorm<kFm>(vpos, p);
        csum[q] = lsum[q] = 0.f;
    }
    PT_USTAMP(sk[0].trace, 1);
    // on-chip accumulators of the positive's rows: aH over the tail-corrupted negatives' dL/dv, aT minus the
    // head-corrupted ones'; the relation's is their difference (with one negative per positive, as in
    // PuTransE, exactly the same sum; not kept live: the 16-float rows spilled with it)
    Vec aH[NP], aT[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        vzero(aH[q]); vzero(aT[q]);
    }
    const float m = P.margin, inv = P.inv_count;
    for (int k = 0; k < neg; ++k) {
        if (!kPrefetch || k > 0) {
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                get_neg(q, k, e[q], tail_side[q]);
                trow<SC1>(x[q], P.ent, P.ent_total, e[q], D, lane);
            }
        }
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            if (nf) vnormalize<kFm>(x[q], x[q]);
#pragma unroll
            for (int i = 0; i < Vec::N; ++i)
                x[q].x[i] = tail_side[q] ? (hh[q].x[i] + rh[q].x[i]) - x[q].x[i] : (x[q].x[i] + rh[q].x[i]) - th[q].x[i];
            const float ns = vpnorm<kFm>(x[q], p);
            PT_USTAMP(sk[0].trace, 2);
            const float a = ps[q] - ns;
            lsum[q] += a > -m ? a : -m;
            const float c = a > -m ? inv : (a == -m ? inv * 0.5f : 0.f);
            if (c != 0.f) {
                csum[q] += c;
                vpnorm_bwd<kFm>(x[q], ns, p, -c, x[q]);   // x := d loss / d v_k
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) {
                    if (tail_side[q]) aH[q].x[i] += x[q].x[i]; else aT[q].x[i] -= x[q].x[i];
                }
                if (tail_side[q]) {
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) x[q].x[i] = -x[q].x[i];
                }
                sk[q].ent(e[q], x[q], D, lane);   // corrupted tail gets -g, corrupted head +g
                PT_USTAMP(sk[0].trace, 3);
            } else if constexpr (ALWAYS) {
                vzero(x[q]);
                sk[q].ent(e[q], x[q], D, lane);
            }
        }
    }
    float loss = 0.f;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
        Vec aR;
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) aR.x[i] = aH[q].x[i] - aT[q].x[i];
        if (csum[q] != 0.f) {
            Vec g;   // the positive's dL/dv, v+ re-formed (same expression as the forward)
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) g.x[i] = (hh[q].x[i] + rh[q].x[i]) - th[q].x[i];
            vpnorm_bwd<kFm>(g, ps[q], p, csum[q], g);
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) {
                aH[q].x[i] += g.x[i];
                aR.x[i] += g.x[i];
                aT[q].x[i] -= g.x[i];
            }
        }
        PT_USTAMP(sk[0].trace, 4);
        // no active pair: every accumulator is zero, nothing to route. Otherwise the three rows go out
        // without a zero test (three lane-group reductions per positive): a row whose sum cancelled to zero
        // is a zero contribution, and a zero gradient leaves a row and its Adagrad state unchanged
        if (csum[q] != 0.f) {
            sk[q].rel(rp[q], aR, D, lane);
            PT_USTAMP(sk[0].trace, 5);
            sk[q].ent(hp[q], aH[q], D, lane);
            PT_USTAMP(sk[0].trace, 6);
            sk[q].ent(tp[q], aT[q], D, lane);
        } else if constexpr (ALWAYS) {   // (no active pair: the accumulators are zero)
            sk[q].rel(rp[q], aR, D, lane);
            sk[q].ent(hp[q], aH[q], D, lane);
            sk[q].ent(tp[q], aT[q], D, lane);
        }
        loss += lsum[q];
    }
    PT_USTAMP(sk[0].trace, 7);
    return loss;
}

// TransH counterpart of transe_step (group_step's TransH algebra with the sampler's one-side negatives):
// the relation, its normal vector and the uncorrupted side are the positive's, kept on chip; the
// projected positive rows are re-formed where the backward needs them instead of being held (the
// universe kernel's register budget). Entity gradients leave raw (projection and normalize Jacobians
// applied here, they depend on the relation), rel in normalized space, norm_vector in n-hat space.
template <int G, int VEC, int KCH, typename Sink, typename NegFn>
__device__ __forceinline__ float transh_step(const StepParams &P, int hp, int rp, int tp, int neg,
                                             NegFn get_neg, const Sink &sink, int lane) {
    using Vec = V<G, VEC, KCH>;
    constexpr bool kFm = uni_fast(G, VEC * KCH);   // hardware sqrt / rcp (see kUF)
    const int D = (int)P.dim;
    const int p = P.p_norm;
    const bool nf = P.norm_flag != 0;
    Vec H, T, rh, nW, hh, th, vpos;
    uload(H, P.ent + hp * D, D, lane);
    uload(T, P.ent + tp * D, D, lane);
    uload(rh, P.rel + rp * D, D, lane);
    uload(nW, P.normv + rp * D, D, lane);
    int e = 0;   // the first negative's row loads with the positive's
    bool tail_side = false;
    Vec X;
    if (neg > 0) {
        get_neg(0, e, tail_side);
        uload(X, P.ent + e * D, D, lane);
    }
    vnormalize<kFm>(nW, nW);
    const float hdot = vdot(H, nW), tdot = vdot(T, nW);
#pragma unroll
    for (int i = 0; i < Vec::N; ++i) {
        hh.x[i] = H.x[i] - hdot * nW.x[i];
        th.x[i] = T.x[i] - tdot * nW.x[i];
    }
    float hn = 0.f, tn = 0.f;
    if (nf) {
        hn = vnormalize<kFm>(hh, hh);
        vnormalize<kFm>(rh, rh);
        tn = vnormalize<kFm>(th, th);
    }
#pragma unroll
    for (int i = 0; i < Vec::N; ++i) vpos.x[i] = (hh.x[i] + rh.x[i]) - th.x[i];
    const float ps = vpnorm<kFm>(vpos, p);
    Vec aH, aT, aR, aW;
    vzero(aH); vzero(aT); vzero(aR); vzero(aW);
    float csum = 0.f, lsum = 0.f;
    const float m = P.margin, inv = P.inv_count;
    for (int k = 0; k < neg; ++k) {
        if (k > 0) {
            get_neg(k, e, tail_side);
            uload(X, P.ent + e * D, D, lane);
        }
        Vec xs, xh, vk;
        const float ed = vdot(X, nW);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) xs.x[i] = X.x[i] - ed * nW.x[i];
        float en = 0.f;
        if (nf) en = vnormalize<kFm>(xs, xh); else xh = xs;
#pragma unroll
        for (int i = 0; i < Vec::N; ++i)
            vk.x[i] = tail_side ? (hh.x[i] + rh.x[i]) - xh.x[i] : (xh.x[i] + rh.x[i]) - th.x[i];
        const float ns = vpnorm<kFm>(vk, p);
        const float a = ps - ns;
        lsum += a > -m ? a : -m;
        const float c = a > -m ? inv : (a == -m ? inv * 0.5f : 0.f);
        if (c == 0.f) continue;
        csum += c;
        vpnorm_bwd<kFm>(vk, ns, p, -c, vk);   // vk := d loss / d v_k
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            aR.x[i] += vk.x[i];
            if (tail_side) aH.x[i] += vk.x[i]; else aT.x[i] -= vk.x[i];
            xh.x[i] = tail_side ? -vk.x[i] : vk.x[i];   // d / d(normalized projected corrupted row)
        }
        Vec gp;
        if (nf) unormalize_bwd<kFm>(xs, en, xh, gp); else gp = xh;
        const float ng = vdot(nW, gp);
        Vec gw;
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            xh.x[i] = gp.x[i] - nW.x[i] * ng;
            gw.x[i] = -(ed * gp.x[i] + ng * X.x[i]);
        }
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) aW.x[i] += gw.x[i];
        sink.ent(e, xh, D, lane);
    }
    if (csum != 0.f) {
        vpnorm_bwd<kFm>(vpos, ps, p, csum, vpos);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            aH.x[i] += vpos.x[i];
            aR.x[i] += vpos.x[i];
            aT.x[i] -= vpos.x[i];
        }
    }
    if (csum == 0.f) return lsum;   // no active pair: every accumulator is zero (see transe_step)
    sink.rel(rp, aR, D, lane);
    // the positive's two entity rows (a lambda over explicit operands, not a loop selecting arrays by
    // index: that would take their addresses and move them to scratch)
    auto finish = [&](const Vec &acc, const Vec &E, float edot, float en, int row) {
        Vec es, gp;
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) es.x[i] = E.x[i] - edot * nW.x[i];
        if (nf) unormalize_bwd<kFm>(es, en, acc, gp); else gp = acc;
        const float ng = vdot(nW, gp);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            es.x[i] = gp.x[i] - nW.x[i] * ng;
            aW.x[i] -= edot * gp.x[i] + ng * E.x[i];
        }
        sink.ent(row, es, D, lane);
    };
    finish(aH, H, hdot, hn, hp);
    finish(aT, T, tdot, tn, tp);
    sink.norm(rp, aW, D, lane);
    return lsum;
}

// Exact x mod d for 64-bit x and a divisor fixed for a universe (its trainTotal, entTotal - 1): one 64 x 64 -> high
// 64 multiply by m = floor((2^64 - 1) / d) estimates the quotient q with floor(x / d) - 2 <= q <= floor(x / d), two
// selects correct the remainder. Replaces the generic 64-bit urem (a long VALU sequence) of rand_max (Random.h:
// 23-25: randd % x) in the presampler, whose draws are otherwise all 64-bit divisions.
struct FastMod {
    uint64_t m, d;
};
__device__ __forceinline__ FastMod fastmod_make(uint64_t d) { return FastMod{d ? ~0ull / d : 0ull, d}; }
__device__ __forceinline__ uint64_t fastmod(uint64_t x, const FastMod &f) {
    const uint64_t q = __umul64hi(x, f.m);
    uint64_t r = x - q * f.d;
    r = r >= f.d ? r - f.d : r;
    r = r >= f.d ? r - f.d : r;
    return r;
}

// The presampler's stream jumps from LDS tables (built once per universe): positive b of sampler call c starts at
// position (c * len + j) * dpp of its thread slice's stream (Base.cpp:200-207: slice id = b / per, j = b - id * per,
// len the slice's size), i.e. LCG^((c * len + j) * dpp) = TC[c][len == per ? 0 : 1] o TJ[j] applied to the slice's
// chunk-start state - two affine maps instead of an O(log n) jump of 64-bit multiplies per draw.
constexpr int kPreJ = 64, kPreC = 32;
struct PreTables {
    Affine j[kPreJ];        // LCG^(j * dpp)
    Affine c[kPreC][2];     // LCG^(c * per * dpp), LCG^(c * rem * dpp) (rem: the last non-empty slice's size)
};

// The presampler of a universe workgroup (every `pchunk` steps): the next nb batches (TrainDataLoader.sampling()
// calls) drawn at once into LDS, lane-parallel - batch j of the chunk is sampler call j after the chunk-start stream
// states - then the streams advanced past them
template <int NT>
__device__ __forceinline__ void presample_draw(int nb, const DeviceGraph &g, uint64_t *s_states,
                                               const PreTables *pre, const FastMod &fm_n, const FastMod &fm_e,
                                               int threads, int bs, int neg, int bern, int filter, int dpp, int per,
                                               int seq, bool fastpre, int32_t *s_bh, int32_t *s_br, int32_t *s_bt) {
    const int tid = threadIdx.x;
    for (int q = tid; q < nb * bs; q += NT) {
        const int s = q / bs, b = q - s * bs;
        if (fastpre && !filter) {
            // the same draws as draw_positive / draw_negative (bit-identical streams and values):
            // table jumps, 32-bit slice arithmetic, rand_max by fastmod
            const int id = b / per, j = b - id * per;
            const PreTables &T = *pre;
            const Affine m1 = T.j[j], m2 = T.c[s][bs - id * per >= per ? 0 : 1];
            uint64_t st = m1.a * s_states[id] + m1.c;
            st = m2.a * st + m2.c;
            const int i = (int)fastmod(lcg_next(st), fm_n);
            i32x4 ra, rc;
            graph_rec(g, i, ra, rc);
            int32_t *bh = s_bh + s * seq, *br = s_br + s * seq, *bt = s_bt + s * seq;
            bh[b] = ra.x; br[b] = ra.y; bt[b] = ra.z;
            const float prob = bern ? g.bern_prob[ra.y] : 500.f;
            for (int k = 0; k < neg; ++k) {
                // coin, then the corruption (Corrupt.h:18-25, 68-74: skips the passed entity)
                const bool tail = (float)(lcg_next(st) % 1000ULL) < prob;
                const int tmp = (int)fastmod(lcg_next(st), fm_e);
                const int skip = tail ? ra.x : ra.z;
                const int e = tmp < skip ? tmp : tmp + 1;
                const int o = (k + 1) * bs + b;
                bh[o] = tail ? ra.x : e;
                bt[o] = tail ? e : ra.z;
                br[o] = ra.y;
            }
            continue;
        }
        const PosDraw pd = draw_positive(g, s_states, threads, bs, b, dpp, s);
        int32_t *bh = s_bh + s * seq, *br = s_br + s * seq, *bt = s_bt + s * seq;
        bh[b] = (int32_t)pd.h; br[b] = (int32_t)pd.r; bt[b] = (int32_t)pd.t;
        for (int k = 0; k < neg; ++k) {
            int side;
            const int e = (int)draw_negative(g, pd, k, bern, filter, &side);
            const int o = (k + 1) * bs + b;
            bh[o] = (int32_t)(side ? pd.h : e);
            bt[o] = (int32_t)(side ? e : pd.t);
            br[o] = (int32_t)pd.r;
        }
    }
    __syncthreads();
    if (tid < threads) {   // the chunk consumed nb calls of the streams
        int len = bs - tid * per;
        len = len < 0 ? 0 : (len > per ? per : len);
        s_states[tid] = lcg_jump(s_states[tid], (uint64_t)len * (uint64_t)dpp * (uint64_t)nb);
    }
}

// Dynamic LDS layout (int32 units; the host sizes it for the largest universe of the launch):
//   list[list_cap] | flags[E + 2R] or [2R] | head[E] + next[ccap] (contrib) |
//   batch h, r, t [3][pchunk * bs * (1 + neg)] (pchunk > 0) | rel (+ norm) gradient rows [R][D] floats
// LDS state of a universe workgroup that is not in the dynamic area (declared once by the kernel)
struct UniShared {
    int32_t *dyn;
    uint64_t *states;   // [64]
    int *count, *ccount;
    float *loss;
    PreTables *pre;
    int *rcount = nullptr;   // (team universes: the step's relation count)
};

// One universe's whole training run (all epochs x nbatches steps) by the calling workgroup.
// PLAN: the LDS plan, fixed at compile time for the two plans the benchmark shapes take (fewer code paths
// in the kernel: its register allocation is for the paths it holds - measured, the general kernel spills
// SGPRs 1.3-1.5x as often and the 16-float class spilled 396 VGPRs against 110):
//   1 = entity rows as contribution lists, relation / norm_vector gradient rows and touched flags in LDS,
//       presampled batches, no agent-scope fences (C3, C4);
//   2 = every row as a contribution list (relation rows too many for LDS: C5), presampled batches;
//   0 = the launch configuration's choices at run time (fallbacks: global float atomics, global flags,
//       per-step sampling).
template <int MODEL, int G, int VEC, int KCH, int NT, int PLAN, bool HOT = false>
__device__ __forceinline__ void universe_run(const UniverseDev &U, int p_norm, int norm_flag, int opt, int neg,
                                             int bern, int filter, const UniverseLaunch &cfg, const UniShared &S) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = NT / G;
    // the first negative's row loaded with the positive's (transe_step's kPrefetch) also for the hot kernels'
    // rows over 128 floats (32 or 64 lanes; r04 same-box A/B: C4 99.4 -> 91.0 ms, its longest universe's phase
    // A 27.9k -> 24.4k cycles/step; for C3's 16-lane hot shapes the set was 1 ms slower, so they do not)
    constexpr bool PF = HOT && G >= 32;
    int32_t *s_dyn = S.dyn;
    uint64_t *s_states = S.states;
    int &s_count = *S.count;
    int &s_ccount = *S.ccount;
    float &s_loss = *S.loss;
    const int tid = threadIdx.x, lane = tid % G, grp = tid / G;
    // 32-bit sizes and indices (a universe is small): half the scalar registers of 64-bit ones, which the
    // kernels spill into VGPR lanes
    const int bs = (int)U.bs, threads = (int)U.threads, D = (int)U.dim;
    const int E = (int)U.g.ent_total, R = (int)U.g.rel_total;
    const bool contrib = PLAN != 0 || (cfg.contrib && U.contrib);
    const int seq = bs * (1 + neg);
    const int nbatches = (int)U.nbatches, epochs = (int)U.epochs;
    const int pchunk = (int)(cfg.pchunk < U.nbatches ? cfg.pchunk : U.nbatches);
    const bool presampled = PLAN != 0 || pchunk > 0;
    const bool agent_fence = PLAN == 0 && cfg.agent_fence;
    const bool lds_flags = PLAN == 1 || (PLAN == 0 && cfg.lds_flags);
    // carve the LDS
    const bool rel_list = PLAN == 2 || (PLAN == 0 && contrib && cfg.rel_list);
    const int ccap = bs * ((rel_list ? 4 : 2) + neg);
    int32_t *p = s_dyn;
    int32_t *s_list = p;
    p += cfg.list_cap;
    int32_t *s_flags = p;   // [E (entity atomics only)][R][R] (relation rows not in lists)
    const int nflags = lds_flags ? ((contrib ? 0 : E) + (rel_list ? 0 : 2 * R)) : 0;
    p += (nflags + 3) & ~3;
    int32_t *s_head = p;
    const int nheads = contrib ? E + 2 * R : 0;
    int32_t *s_next = p + ((nheads + 3) & ~3);
    if (contrib) p += ((nheads + 3) & ~3) + ((ccap + 3) & ~3);
    int32_t *s_bh = p, *s_br = p + pchunk * seq, *s_bt = p + 2 * pchunk * seq;
    p += 3 * pchunk * seq;
    float *s_grel = reinterpret_cast<float *>(p);
    const int nrelg = (PLAN == 1 || (PLAN == 0 && cfg.lds_relgrad)) && !rel_list ? R * D * (MODEL == 1 ? 2 : 1) : 0;

    if (tid < threads) s_states[tid] = U.states[tid];
    // presampler jump tables (PreTables): positives per thread slice `per`, the last non-empty slice's size `rem`
    const int per = bs % threads == 0 ? bs / threads : bs / threads + 1;
    const int rem = per > 0 ? bs - (bs / per) * per : 0;
    const int dpp = 1 + 2 * neg;
    const bool fastpre = presampled && per <= kPreJ && pchunk <= kPreC;
    if (fastpre) {
        PreTables &T = *S.pre;
        if (tid < kPreJ) {
            T.j[tid] = lcg_power((uint64_t)tid * (uint64_t)dpp);
        } else if (tid < kPreJ + 2 * kPreC) {
            const int c = (tid - kPreJ) >> 1, w = (tid - kPreJ) & 1;
            T.c[c][w] = lcg_power((uint64_t)c * (uint64_t)(w ? rem : per) * (uint64_t)dpp);
        }
    }
    const FastMod fm_n = fastmod_make((uint64_t)U.g.train_total), fm_e = fastmod_make((uint64_t)(E - 1));
    for (int i = tid; i < nflags; i += NT) s_flags[i] = 0;
    for (int i = tid; i < nheads; i += NT) s_head[i] = -1;
    for (int i = tid; i < nrelg; i += NT) s_grel[i] = 0.f;
    StepParams P{};
    P.model = MODEL; P.p_norm = p_norm; P.norm_flag = norm_flag; P.opt = opt;
    P.lr = U.lr; P.margin = U.margin;
    P.ent_total = E; P.rel_total = R; P.dim = D;
    P.ent = U.ent; P.rel = U.rel; P.normv = U.normv;
    P.ent_acc = U.ent_acc; P.rel_acc = U.rel_acc; P.norm_acc = U.norm_acc;
    P.batch_size = bs; P.neg = neg;
    P.inv_count = 1.0f / (float)(bs * neg);
    UniverseSink<PLAN> sink{U.gent, U.grel, U.gnorm, U.fent, U.frel, U.fnorm, s_list, &s_count,
                      contrib ? U.contrib : nullptr, s_head, s_next, &s_ccount, E, R, rel_list};
    if (lds_flags) {
        int32_t *f = s_flags;
        if (!contrib) {
            sink.fent = f;
            f += E;
        }
        if (!rel_list) {
            sink.frel = f;
            sink.fnorm = f + R;
        }
    }
    if (nrelg) {
        sink.grel = s_grel;
        sink.gnorm = s_grel + R * D;
    }
    const DeviceGraph &g = U.g;
    float epoch_loss = 0.f;
    uint64_t t_pre = 0, t_a = 0, t_b = 0, t0 = 0;
    const uint64_t w_start = U.prof ? wall_clock64() : 0;   // (100 MHz wall clock: the set's schedule)
    __syncthreads();
    for (int epoch = 0; epoch < epochs; ++epoch) {
        for (int step = 0; step < nbatches; ++step) {
            if (U.prof) t0 = clock64();
            // tuning build: stamps of step 5 of epoch 1 (phase A rounds [8 + 8r, +8), phase B rounds [48 + r])
            uint64_t *const tr = U.prof && epoch == 1 && step == 5 && grp == 0 ? U.prof : nullptr;
            const int cs = pchunk > 0 ? step % pchunk : 0;
            if (presampled && cs == 0) {
                // the next min(pchunk, left) batches drawn at once into LDS: batch j of the chunk is
                // sampler call j after the chunk-start stream states (presample_draw's draws, written out here:
                // as a call the class kernels' allocation spills more, round 6)
                const int nb = nbatches - step < pchunk ? nbatches - step : pchunk;
                for (int q = tid; q < nb * bs; q += NT) {
                    const int s = q / bs, b = q - s * bs;
                    if (fastpre && !filter) {
                        // the same draws as draw_positive / draw_negative (bit-identical streams and values):
                        // table jumps, 32-bit slice arithmetic, rand_max by fastmod
                        const int id = b / per, j = b - id * per;
                        const PreTables &T = *S.pre;
                        const Affine m1 = T.j[j], m2 = T.c[s][bs - id * per >= per ? 0 : 1];
                        uint64_t st = m1.a * s_states[id] + m1.c;
                        st = m2.a * st + m2.c;
                        const int i = (int)fastmod(lcg_next(st), fm_n);
                        i32x4 ra, rc;
                        graph_rec(g, i, ra, rc);
                        int32_t *bh = s_bh + s * seq, *br = s_br + s * seq, *bt = s_bt + s * seq;
                        bh[b] = ra.x; br[b] = ra.y; bt[b] = ra.z;
                        const float prob = bern ? g.bern_prob[ra.y] : 500.f;
                        for (int k = 0; k < neg; ++k) {
                            // coin, then the corruption (Corrupt.h:18-25, 68-74: skips the passed entity)
                            const bool tail = (float)(lcg_next(st) % 1000ULL) < prob;
                            const int tmp = (int)fastmod(lcg_next(st), fm_e);
                            const int skip = tail ? ra.x : ra.z;
                            const int e = tmp < skip ? tmp : tmp + 1;
                            const int o = (k + 1) * bs + b;
                            bh[o] = tail ? ra.x : e;
                            bt[o] = tail ? e : ra.z;
                            br[o] = ra.y;
                        }
                        continue;
                    }
                    const PosDraw pd = draw_positive(g, s_states, threads, bs, b, dpp, s);
                    int32_t *bh = s_bh + s * seq, *br = s_br + s * seq, *bt = s_bt + s * seq;
                    bh[b] = (int32_t)pd.h; br[b] = (int32_t)pd.r; bt[b] = (int32_t)pd.t;
                    for (int k = 0; k < neg; ++k) {
                        int side;
                        const int e = (int)draw_negative(g, pd, k, bern, filter, &side);
                        const int o = (k + 1) * bs + b;
                        bh[o] = (int32_t)(side ? pd.h : e);
                        bt[o] = (int32_t)(side ? e : pd.t);
                        br[o] = (int32_t)pd.r;
                    }
                }
                __syncthreads();
                if (tid < threads) {   // the chunk consumed nb calls of the streams
                    int len = bs - tid * per;
                    len = len < 0 ? 0 : (len > per ? per : len);
                    s_states[tid] = lcg_jump(s_states[tid], (uint64_t)len * (uint64_t)dpp * (uint64_t)nb);
                }
            }
            if (tid == 0) {
                s_count = 0;
                s_ccount = 0;
                s_loss = 0.f;
            }
            phase_barrier(agent_fence);
            if (U.prof) {
                const uint64_t t1 = clock64();
                t_pre += t1 - t0;
                t0 = t1;
            }
            PT_USTAMP(tr, 46);
            // ---- phase A: forward + backward of the step's positives
            float lacc = 0.f;   // this lane group's positives' loss, one LDS add per step
            for (int b = grp; b < bs; b += GPB) {
                float lsum;
                sink.slot = (int)(b * ((rel_list ? 4 : 2) + neg));
                sink.trace = tr && b / GPB < 4 ? tr + 8 + 8 * (b / GPB) : nullptr;
                if (presampled) {
                    const int32_t *bh = s_bh + cs * seq, *br = s_br + cs * seq, *bt = s_bt + cs * seq;
                    const int hp = bh[b], rp = br[b], tp = bt[b];
                    if constexpr (MODEL == 0) {
                        // a negative shares one side with its positive: the head when the tail was
                        // corrupted (if both sides match, the negative equals the positive and either
                        // reading gives the same gradients)
                        const int hq[1] = {hp}, rq[1] = {rp}, tq[1] = {tp};
                        const UniverseSink<PLAN> sk[1] = {sink};
                        lsum = transe_step<1, G, VEC, KCH, PF>(
                            P, hq, rq, tq, neg,
                            [&](int, int k, int &e, bool &tail_side) {
                                const int o = (k + 1) * bs + b;
                                tail_side = bh[o] == hp;
                                e = tail_side ? bt[o] : bh[o];
                            },
                            sk, lane);
                    } else {
                        lsum = transh_step<G, VEC, KCH>(
                            P, hp, rp, tp, neg,
                            [&](int k, int &e, bool &tail_side) {
                                const int o = (k + 1) * bs + b;
                                tail_side = bh[o] == hp;
                                e = tail_side ? bt[o] : bh[o];
                            },
                            sink, lane);
                    }
                } else {
                    const PosDraw pd = draw_positive(g, s_states, threads, bs, b, dpp);
                    if constexpr (MODEL == 0) {
                        const int hq[1] = {(int)pd.h}, rq[1] = {(int)pd.r}, tq[1] = {(int)pd.t};
                        const UniverseSink<PLAN> sk[1] = {sink};
                        lsum = transe_step<1, G, VEC, KCH, PF>(
                            P, hq, rq, tq, neg,
                            [&](int, int k, int &e, bool &tail_side) {
                                int side;
                                e = (int)draw_negative(g, pd, k, bern, filter, &side);
                                tail_side = side != 0;
                            },
                            sk, lane);
                    } else {
                        lsum = transh_step<G, VEC, KCH>(
                            P, (int)pd.h, (int)pd.r, (int)pd.t, neg,
                            [&](int k, int &e, bool &tail_side) {
                                int side;
                                e = (int)draw_negative(g, pd, k, bern, filter, &side);
                                tail_side = side != 0;
                            },
                            sink, lane);
                    }
                }
                lacc += lsum;
            }
            if (lane == 0 && grp < bs) atomicAdd(&s_loss, lacc);
            phase_barrier(agent_fence);
            if (U.prof) {
                const uint64_t t1 = clock64();
                t_a += t1 - t0;
                t0 = t1;
            }
            // ---- phase B: row updates of the touched rows, RB rows per lane group at a time (all their
            // loads in flight together: the pass is a chain of dependent memory round trips otherwise)
            const int n = s_count;
            // (TransH: 2 rows of 8 floats per lane in flight spill its step's registers; TransE keeps 2)
            // (1024-thread workgroups: half the rows per lane group, twice the lane groups; 128 VGPRs per lane)
            // (r04: two rows per lane group in the hot kernels' 5-6-float shapes spill 28-68 B per lane, phase B
            // of C3's D = 69 universe 5.9k -> 8.2k cycles per step)
            // (r04: the hot kernels' phase B on lane groups of half the width - twice the floats per lane, twice the
            // rows per round: phase B of C3's D = 68 universe 4.3k -> 14.2k, of C4's longest 23k -> 89k cycles per step)
            constexpr int RB = VEC * KCH >= 16 ? 1 : (VEC * KCH > 4 ? (MODEL == 1 || NT > 512 ? 1 : 2) : (NT > 512 ? 2 : 4));
            constexpr bool kFastUpd = uni_fast(G, VEC * KCH);
            // (guards, not breaks, inside the unrolled loops: the row arrays must stay in registers)
            PT_USTAMP(tr, 47);
            for (int i0 = grp * RB; i0 < n; i0 += GPB * RB) {
                if (i0 / (GPB * RB) < 14) PT_USTAMP(tr, 48 + i0 / (GPB * RB));
                Vec x[RB], gs[RB], a[RB], y[RB];
                int32_t code[RB], c1[RB];
#pragma unroll
                for (int u = 0; u < RB; ++u) {
                    code[u] = i0 + u < n ? s_list[i0 + u] : -1;
                    c1[u] = -1;
                    if (code[u] >= 0) {
                        const int table = code[u] & 3;
                        const int row = code[u] >> 2;
                        const float *wp = (table == 0 ? U.ent : (table == 1 ? U.rel : U.normv)) + row * D;
                        const float *ap = (table == 0 ? U.ent_acc : (table == 1 ? U.rel_acc : U.norm_acc)) + row * D;
                        uload(x[u], wp, (int)D, lane);
                        if (opt != 0) uload(a[u], ap, (int)D, lane);
                        if ((table == 0 && contrib) || (table > 0 && rel_list)) {
                            // the row's contributions (linked in LDS): the first two loads issued with the
                            // row's own, the rest walked below; summed in list order
                            const int32_t c0 = s_head[(table == 0 ? 0 : (table == 1 ? E : E + R)) + row];
                            uload(gs[u], U.contrib + c0 * D, (int)D, lane);
                            c1[u] = s_next[c0];
                            if (c1[u] >= 0) uload(y[u], U.contrib + c1[u] * D, (int)D, lane);
                        } else {
                            vload(gs[u], (table == 0 ? sink.gent : (table == 1 ? sink.grel : sink.gnorm)) + row * D,
                                  (int)D, lane);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < RB; ++u) {
                    if (code[u] >= 0 && c1[u] >= 0) {
#pragma unroll
                        for (int j = 0; j < Vec::N; ++j) gs[u].x[j] += y[u].x[j];
                        if constexpr (PLAN == 2) {   // (the relation rows' long lists, four rows in flight)
                            list_sum<PT_UNI_LIST_BATCH>(gs[u], s_next[c1[u]], s_next, [&](Vec &r, int32_t c) {
                                uload(r, U.contrib + c * D, (int)D, lane);
                            });
                        } else {
                            for (int32_t c = s_next[c1[u]]; c >= 0; c = s_next[c]) {
                                uload(y[u], U.contrib + c * D, (int)D, lane);
#pragma unroll
                                for (int j = 0; j < Vec::N; ++j) gs[u].x[j] += y[u].x[j];
                            }
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < RB; ++u) {
                    if (code[u] < 0) continue;
                    const int table = code[u] & 3;
                    const int row = code[u] >> 2;
                    float *wp = (table == 0 ? U.ent : (table == 1 ? U.rel : U.normv)) + row * D;
                    float *ap = (table == 0 ? U.ent_acc : (table == 1 ? U.rel_acc : U.norm_acc)) + row * D;
                    // ent rows of TransE and every rel / norm_vector row carry normalized-space gradients
                    const bool jac = table == 0 ? (MODEL == 0 && norm_flag) : (table == 1 ? norm_flag != 0 : true);
                    Vec gg;
                    if (jac) {
                        const float nx = fsqrt<kFastUpd>(vdot(x[u], x[u]));
                        unormalize_bwd<kFastUpd>(x[u], nx, gs[u], gg);
                    } else {
                        gg = gs[u];
                    }
                    if (opt == 0) {
#pragma unroll
                        for (int j = 0; j < Vec::N; ++j) x[u].x[j] = x[u].x[j] + (-U.lr) * gg.x[j];
                    } else {
#pragma unroll
                        for (int j = 0; j < Vec::N; ++j) {
                            a[u].x[j] = a[u].x[j] + gg.x[j] * gg.x[j];
                            if constexpr (kFastUpd)
                                x[u].x[j] = x[u].x[j] + (-U.lr) * (gg.x[j] * frcp<true>(fsqrt<true>(a[u].x[j]) + 1e-10f));
                            else
                                x[u].x[j] = x[u].x[j] + (-U.lr) * gg.x[j] / (sqrtf(a[u].x[j]) + 1e-10f);
                        }
                        ustore(a[u], ap, (int)D, lane);
                    }
                    ustore(x[u], wp, (int)D, lane);
                    if ((table == 0 && contrib) || (table > 0 && rel_list)) {
                        if (lane == 0) s_head[(table == 0 ? 0 : (table == 1 ? E : E + R)) + row] = -1;
                    } else {
                        Vec z;
                        vzero(z);
                        vstore(z, (table == 0 ? sink.gent : (table == 1 ? sink.grel : sink.gnorm)) + row * D, (int)D,
                               lane);
                        if (lane == 0) (table == 0 ? sink.fent : (table == 1 ? sink.frel : sink.fnorm))[row] = 0;
                    }
                }
            }
            if (!presampled && tid < threads) {   // the step consumed bs positives x dpp draws
                int len = bs - tid * per;
                len = len < 0 ? 0 : (len > per ? per : len);
                s_states[tid] = lcg_jump(s_states[tid], (uint64_t)len * (uint64_t)dpp);
            }
            if (tid == 0) epoch_loss += s_loss * P.inv_count + U.margin;
            if (U.prof) {
                const uint64_t t1 = clock64();
                t_b += t1 - t0;
                PT_USTAMP(tr, 63);
            }
        }
        if (tid == 0 && U.losses) U.losses[epoch] = epoch_loss;
        epoch_loss = 0.f;
    }
    phase_barrier(agent_fence);
    if (U.prof && tid == 0) {
        U.prof[0] = t_pre;
        U.prof[1] = t_a;
        U.prof[2] = t_b;
        U.prof[3] = (uint64_t)U.epochs * U.nbatches;
        U.prof[4] = (uint64_t)bs;
        U.prof[5] = (uint64_t)D;
        U.prof[6] = (uint64_t)E;
        // the universe's start on the 100 MHz wall clock (low 32 bits) and its duration in those ticks
        U.prof[7] = (w_start << 32) | ((wall_clock64() - w_start) & 0xffffffffull);
        // where the workgroup ran: XCD (HW_REG_XCC_ID) and HW_REG_HW_ID (SE / SH / CU / SIMD / wave fields)
        U.prof[63] = ((uint64_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32) |
                     (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
    if (tid < threads) U.states[tid] = s_states[tid];
}

// row shapes of the universe kernel: narrower lane groups than the single-model kernels (2 x VEC=4
// or 4 x VEC=1 chunks per lane) so a step's ~25-100 positives and ~100-300 touched rows take few rounds
#define PT_USHAPES(X)                                                                                  \
    X(0, 2, 4, 1) X(1, 2, 4, 2) X(2, 4, 4, 2) X(3, 8, 4, 2) X(4, 16, 4, 2) X(5, 32, 4, 2) X(6, 64, 4, 2) \
    X(7, 2, 1, 1) X(8, 2, 1, 2) X(9, 2, 1, 4) X(10, 4, 1, 4) X(11, 8, 1, 4) X(12, 16, 1, 4)              \
    X(13, 32, 1, 4) X(14, 64, 1, 4) X(15, 64, 1, 8)                                                      \
    X(16, 2, 4, 4) X(17, 4, 4, 4) X(18, 8, 4, 4) X(19, 16, 4, 4) X(20, 32, 4, 4) X(21, 64, 4, 4)        \
    X(22, 2, 1, 8) X(23, 4, 1, 8) X(24, 8, 1, 8) X(25, 16, 1, 8) X(26, 32, 1, 8)                       \
    X(27, 16, 1, 5) X(28, 16, 1, 6) X(29, 16, 1, 7) X(30, 8, 1, 5) X(31, 8, 1, 6) X(32, 8, 1, 7)        \
    X(33, 4, 1, 5) X(34, 4, 1, 6) X(35, 4, 1, 7) X(36, 2, 4, 3) X(37, 4, 4, 3) X(38, 8, 4, 3)           \
    X(39, 4, 1, 3) X(40, 8, 1, 3) X(41, 16, 1, 3)

// shape class (one kernel each): 0 = at most 4 floats per lane, 1 = 8, 2 = 16 (TransE's wide shapes). (Measured
// r04 and removed: splitting class 1 into 5-6 and 7-8 floats, so the 5-6 kernel - C3's longest universes, 65-96
// dims over 16 lanes - fits 1,024 threads without spilling: C3 52.3 -> 52.8 ms, the fourth launch costs more;
// splitting it by vector width, scalar and float4 rows: C3 40.3 -> 41.1 ms.)
#define PT_UCLASS(V_, K_) ((V_) * (K_) <= 4 ? 0 : ((V_) * (K_) <= 8 ? 1 : 2))

// whether pick_universe_shape can return (G, VEC, KCH) for the model (TransE: wide shapes, TransH: narrow):
// with p chunks per lane, a group of more than 2 and fewer than 64 lanes holds exactly p, the 2-lane group
// up to p and the 64-lane group p or more. Each class kernel compiles only these shapes (fewer paths, a
// register allocation for fewer of them); TransH rows above 512 floats (class 2) are not supported.
constexpr bool shape_reachable(int model, int G, int VEC, int KCH) {
    // (exact_kch_shape: G in (2, 64), so the 2-lane VEC=4 exact shape is the KCH <= p case below)
    const int p = universe_chunks_per_lane(model, VEC);
    if (model == 1 && VEC * KCH > 8) return false;
    if (G > 2 && G < 64 && KCH > p / 2 && KCH < p) return exact_kch_shape(G, VEC);   // see pick_universe_shape
    return G == 2 ? KCH <= p : (G == 64 ? KCH >= p : KCH == p);
}

// Persistent work-queue kernel of one shape CLASS (rows of <= 4 floats per lane, or wider): a workgroup
// takes universes (all of this class, in the host's longest-first order) from an atomic counter until
// the queue is empty - greedy longest-processing-time list scheduling over the launch's workgroups -
// and runs each with its shape's code path. Two classes instead of one kernel for every shape: each
// kernel is register-allocated for its own widest shape (one kernel over all shapes spills the narrow
// ones' state too), and two launches still run concurrently (a launch per shape would need more
// hardware queues than a process gets).
template <int MODEL, int NT, int WPE, int CLS, int PLAN>
__global__ __launch_bounds__(NT, WPE) void k_universes(const UniverseDev *__restrict__ us, int64_t n,
                                                       int *__restrict__ next_universe, int p_norm, int norm_flag,
                                                       int opt, int64_t neg, int bern, int filter,
                                                       UniverseLaunch cfg) {
    extern __shared__ int32_t s_dyn[];
    __shared__ uint64_t s_states[64];
    __shared__ int s_count, s_ccount, s_u;
    __shared__ float s_loss;
    __shared__ PreTables s_pre;
    const UniShared S{s_dyn, s_states, &s_count, &s_ccount, &s_loss, &s_pre};
    for (;;) {
        if (threadIdx.x == 0) s_u = atomicAdd(next_universe, 1);
        __syncthreads();
        // uniform: readfirstlane makes the descriptor loads below scalar (its fields live in SGPRs, not in
        // the VGPRs the step's rows need)
        const int64_t u = __builtin_amdgcn_readfirstlane(s_u);
        __syncthreads();
        if (u >= n) break;   // every wave of the workgroup reads the same u: the whole group exits
        // the 16-float class reads the descriptor's fields where they are used (fewer live scalars: C4 113 ->
        // 104 ms); the narrower classes keep a register copy (C3 65 vs 68 ms)
        const UniverseDev Uc = CLS == 2 ? UniverseDev{} : us[u];
        const UniverseDev &U = CLS == 2 ? us[u] : Uc;
        switch (U.shape) {
#define PT_URUN(ID_, G_, V_, K_)                                                                       \
    case ID_:                                                                                          \
        if constexpr ((CLS < kUniHotBase ? PT_UCLASS(V_, K_) == CLS : ID_ == CLS - kUniHotBase) &&     \
                      shape_reachable(MODEL, G_, V_, K_))                                               \
            universe_run<MODEL, G_, V_, K_, NT, PLAN, (CLS >= kUniHotBase)>(U, p_norm, norm_flag, opt, \
                                                                                   (int)neg, bern, filter, cfg, S); \
        break;
            PT_USHAPES(PT_URUN)
#undef PT_URUN
            default:
                break;
        }
        __syncthreads();
    }
}

}  // namespace dev

namespace detail {
template <int MODEL, int WPE, int CLS, int PLAN, int HOT_G = 0>
hipError_t launch_q(const UniverseDev *d_us, int64_t n, int *counter, int64_t cus, int p_norm, int norm_flag, int opt,
                    int64_t neg, int bern, int filter, const UniverseLaunch &cfg, hipStream_t st) {
    // (a hot single-shape kernel runs a class-1 shape: that class's workgroup size, or universe_hot_threads)
    constexpr int NT = CLS < kUniHotBase ? universe_class_threads(MODEL, CLS) : universe_hot_threads(HOT_G);
    auto kern = dev::k_universes<MODEL, NT, WPE * NT / 512, CLS, PLAN>;
    if (cfg.lds_bytes > (64 << 10)) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)cfg.lds_bytes);
        if (e != hipSuccess) return e;
    }
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(kern), NT,
                                                                (size_t)cfg.lds_bytes);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    int64_t grid = cus * per_cu;
    if (grid > n) grid = n;
    if (grid < 1) grid = 1;
    e = hipMemsetAsync(counter, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), (size_t)cfg.lds_bytes, st, d_us, n, counter, p_norm,
                       norm_flag, opt, neg, bern, filter, cfg);
    return hipGetLastError();
}
}  // namespace detail

// the persistent launch of one shape class under LDS plan PLAN (see universe_run)
template <int PLAN>
hipError_t launch_universes_plan(const UniverseDev *d_us, int64_t n, int *counter, int cls, int64_t cus, int model,
                                 int p_norm, int norm_flag, int opt, int64_t neg, int bern, int filter,
                                 const UniverseLaunch &cfg, hipStream_t st) {
    using detail::launch_q;
    if (cls >= kUniHotBase) {
        // a hot shape's own kernel (plans 1 and 2, TransE); otherwise its universes run in their class kernel
        if constexpr (PLAN != 0) {
            if (model == 0) {
                switch (cls - kUniHotBase) {
#define PT_UHOT(ID_, G_, V_, K_)                                                                                  \
    case ID_:                                                                                                      \
        if constexpr (PT_UCLASS(V_, K_) == 1 && dev::shape_reachable(0, G_, V_, K_))                                \
            return launch_q<0, 2, kUniHotBase + ID_, PLAN, G_>(d_us, n, counter, cus, p_norm, norm_flag, opt, neg,  \
                                                              bern, filter, cfg, st);                                \
        break;
                    PT_USHAPES(PT_UHOT)
#undef PT_UHOT
                    default:
                        break;
                }
            }
        }
        cls = 1;
    }
    if (cls == 0)
        return model == 0 ? launch_q<0, 2, 0, PLAN>(d_us, n, counter, cus, p_norm, norm_flag, opt, neg, bern, filter, cfg, st)
                          : launch_q<1, 2, 0, PLAN>(d_us, n, counter, cus, p_norm, norm_flag, opt, neg, bern, filter, cfg, st);
    if (cls == 1)
        return model == 0 ? launch_q<0, 2, 1, PLAN>(d_us, n, counter, cus, p_norm, norm_flag, opt, neg, bern, filter, cfg, st)
                          : launch_q<1, 2, 1, PLAN>(d_us, n, counter, cus, p_norm, norm_flag, opt, neg, bern, filter, cfg, st);
    if (model == 0)
        return launch_q<0, 2, 2, PLAN>(d_us, n, counter, cus, p_norm, norm_flag, opt, neg, bern, filter, cfg, st);
    return hipErrorInvalidValue;   // TransH universes use the narrow shapes
}
extern template hipError_t launch_universes_plan<1>(const UniverseDev *, int64_t, int *, int, int64_t, int, int, int,
                                                    int, int64_t, int, int, const UniverseLaunch &, hipStream_t);
extern template hipError_t launch_universes_plan<2>(const UniverseDev *, int64_t, int *, int, int64_t, int, int, int,
                                                    int, int64_t, int, int, const UniverseLaunch &, hipStream_t);

}  // namespace pt
