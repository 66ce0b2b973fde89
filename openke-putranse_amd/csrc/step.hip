// HIP kernels of the training step (TransE / TransH forward + backward, gradient routing) for gfx950.
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

// ---------------------------------------------------------------- fused step -----------------
// Gradient sink of the single-model path: memory-side float atomics into per-table gradient rows,
// plus a touched-row flag for the sparse apply pass.
struct GlobalSink {
    float *gent, *grel, *gnorm;
    int *fent, *frel, *fnorm;
    float *lpart;   // per-positive loss partials
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void ent(int64_t row, const V<G, VEC, KCH> &g, int D, int lane) const {
        vatomic(g, gent + row * D, D, lane);
        if (lane == 0) fent[row] = 1;
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void rel(int64_t row, const V<G, VEC, KCH> &g, int D, int lane) const {
        vatomic(g, grel + row * D, D, lane);
        if (lane == 0) frel[row] = 1;
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void norm(int64_t row, const V<G, VEC, KCH> &g, int D, int lane) const {
        vatomic(g, gnorm + row * D, D, lane);
        if (lane == 0) fnorm[row] = 1;
    }
};

// General step on an externally given batch (Trainer.train_one_step): any (h, r, t) per slot.
template <int MODEL, int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_step(StepParams P, const int64_t *__restrict__ bh,
                                              const int64_t *__restrict__ bt, const int64_t *__restrict__ br,
                                              GlobalSink sink, float *__restrict__ loss) {
    constexpr int GPB = 256 / G;
    const int lane = threadIdx.x % G;
    const int64_t bs = P.batch_size, neg = P.neg;
    const int64_t b = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    if (b >= bs) return;
    const int64_t hp = bh[b], tp = bt[b], rp = br[b];
    const float lsum = group_step<MODEL, G, VEC, KCH>(
        P, hp, rp, tp, neg,
        [&](int64_t k, int64_t &h, int64_t &t, int64_t &r) {
            const int64_t o = (k + 1) * bs + b;
            h = bh[o]; t = bt[o]; r = br[o];
        },
        sink, lane);
    if (lane == 0 && sink.lpart) sink.lpart[b] = lsum;
}

// Fused step with in-kernel sampling (the Trainer.run hot loop).
//
// A positive is owned by S lane groups ("sub-groups"); sub-group s takes negatives
// [s*nper, min(neg, (s+1)*nper)). Each sub-group draws its negatives lane-parallel into LDS, then
// loads EVERY row it needs before its first gradient store/atomic (s_waitcnt vmcnt counts loads,
// stores and atomics in issue order, so a load queued behind an atomic would wait for it), keeping up
// to NCH negative rows in registers. The positive's forward is recomputed by every sub-group (its
// rows are L1/L2 hits); the positive-row gradient partials meet in LDS and sub-group 0 finishes them.
// Rows use the VEC=1 layout, so each atomic/store wave-instruction covers 64 contiguous floats.
//
// CSR = true: the batch was drawn by k_sample_csr; the corrupted entities' gradient rows are written
// with plain stores to their counting-sort slots (contrib) instead of float atomics.
template <int MODEL, int G, int VEC, int KCH, int NCH, int S, bool CSR, bool DB>
__global__ __launch_bounds__(256) void k_step_sampled(StepParams P, DeviceGraph g, const uint64_t *__restrict__ states,
                                                      int64_t threads, int bern, int filter, GlobalSink sink,
                                                      float *__restrict__ loss, CsrWork cw) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;      // lane groups per block
    constexpr int PPB = GPB / S;      // positives per block
    constexpr int RW = KCH * G * VEC; // floats per row slot in the reduction area
    // LDS: s_neg[PPB*neg] (entity << 1 | tail_side) [, s_dst[PPB*neg]] , then red[GPB][4][RW] + cs[GPB][2]
    extern __shared__ __attribute__((aligned(16))) int64_t s_neg[];
    const int lane = threadIdx.x % G;
    const int grp = threadIdx.x / G;
    const int pl = grp / S;            // positive slot in the block
    const int sub = grp % S;
    const int64_t bs = P.batch_size, neg = P.neg;
    const int64_t b = (int64_t)blockIdx.x * PPB + pl;
    const bool active = b < bs;
    const int64_t nper = (neg + S - 1) / S;
    const int64_t k_lo = sub * nper < neg ? sub * nper : neg;
    const int64_t k_hi = k_lo + nper < neg ? k_lo + nper : neg;
    int64_t *s_dst = s_neg + PPB * neg;
    float *red = reinterpret_cast<float *>(s_neg + PPB * neg * (CSR ? 2 : 1));
    float *cs = red + GPB * 4 * RW;
    PosDraw pd{};
    const int D = (int)P.dim;
    Vec H, T, Rr, W, nW, hh, th, rh, vpos;
    if (active) {
        if constexpr (!CSR) {
            pd = draw_positive(g, states, threads, bs, b, 1 + 2 * neg);
        } else {
            const int4 q = cw.pos[b];
            pd.h = q.x; pd.r = q.y; pd.t = q.z;
        }
        pd.h = uni<G>((int32_t)pd.h); pd.r = uni<G>((int32_t)pd.r); pd.t = uni<G>((int32_t)pd.t);
        // the positive's rows are in flight while the negatives are drawn / fetched
        vload(H, P.ent + pd.h * D, D, lane);
        vload(T, P.ent + pd.t * D, D, lane);
        vload(Rr, P.rel + pd.r * D, D, lane);
        if constexpr (MODEL == 1) vload(W, P.normv + pd.r * D, D, lane);
        if constexpr (!CSR) {
            for (int64_t k = k_lo + lane; k < k_hi; k += G) {
                int side;
                const int64_t e = draw_negative(g, pd, k, bern, filter, &side);
                s_neg[pl * neg + k] = (e << 1) | side;
            }
        } else {
            for (int64_t k = k_lo + lane; k < k_hi; k += G) {
                s_neg[pl * neg + k] = cw.neg[b * neg + k];
                const int32_t r = cw.off[b * neg + k];   // destination, or rank in the bucket (rank_only)
                s_dst[pl * neg + k] = cw.rank_only ? r + cw.start[cw.neg[b * neg + k] >> 1] : r;
            }
        }
    }
    __syncthreads();
    const int p = P.p_norm;
    const bool nf = P.norm_flag != 0;
    const int64_t hp = pd.h, rp = pd.r, tp = pd.t;
    const int64_t *mine = s_neg + pl * neg;
    // DB: double buffer (the next chunk's rows load while this chunk computes), for nper > NCH
    Vec EA[NCH], EB[DB ? NCH : 1];
    Vec aH, aT, aR, aW;
    vzero(aH); vzero(aT); vzero(aR); vzero(aW);
    float csum = 0.f, lsum = 0.f;
    Vec Hs, Ts;
    float hn = 0, tn = 0, hdot = 0, tdot = 0, ps = 0;
    if (active) {
        auto load_chunk = [&](Vec(&E)[NCH], int64_t c0) {
#pragma unroll
            for (int k = 0; k < NCH; ++k)
                if (c0 + k < k_hi && !PT_ABLATE(P.dbg, 4)) vload(E[k], P.ent + (mine[c0 + k] >> 1) * D, D, lane);
        };
        load_chunk(EA, k_lo);
        // ---- positive forward
        Hs = H; Ts = T;
        if constexpr (MODEL == 1) {
            vnormalize<true>(W, nW);
            hdot = vdot(H, nW);
            tdot = vdot(T, nW);
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) {
                Hs.x[i] = H.x[i] - hdot * nW.x[i];
                Ts.x[i] = T.x[i] - tdot * nW.x[i];
            }
        }
        if (nf) {
            hn = vnormalize<true>(Hs, hh);
            vnormalize<true>(Rr, rh);
            tn = vnormalize<true>(Ts, th);
        } else {
            hh = Hs; rh = Rr; th = Ts;
        }
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) vpos.x[i] = (hh.x[i] + rh.x[i]) - th.x[i];
        ps = vpnorm<true>(vpos, p);
        const float m = P.margin, inv = P.inv_count;
        auto process = [&](Vec(&E)[NCH], int64_t c0) {
#pragma unroll
            for (int k = 0; k < NCH; ++k) {
                if (c0 + k >= k_hi) return;
                const int32_t v = uni<G>((int32_t)mine[c0 + k]);
                const int64_t e = v >> 1;
                const bool tail_side = v & 1;
                Vec Es = E[k], eh, vk;
                float ed = 0.f, en = 0.f;
                if constexpr (MODEL == 1) {
                    ed = vdot(E[k], nW);
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) Es.x[i] = E[k].x[i] - ed * nW.x[i];
                }
                if (nf) en = vnormalize<true>(Es, eh); else eh = Es;
#pragma unroll
                for (int i = 0; i < Vec::N; ++i)
                    vk.x[i] = tail_side ? (hh.x[i] + rh.x[i]) - eh.x[i] : (eh.x[i] + rh.x[i]) - th.x[i];
                const float ns = vpnorm<true>(vk, p);
                const float a = uni<G>(ps - ns);
                lsum += a > -m ? a : -m;
                const float c = a > -m ? inv : (a == -m ? inv * 0.5f : 0.f);
                float *dst = nullptr;
                if constexpr (CSR) dst = cw.contrib + (int64_t)uni<G>((int32_t)s_dst[pl * neg + c0 + k]) * D;
                if (c == 0.f) {
                    if constexpr (CSR) {   // the reserved slot must still be defined
                        Vec z;
                        vzero(z);
                        vstore(z, dst, D, lane);
                    }
                    continue;
                }
                csum += c;
                Vec gk, gs;
                vpnorm_bwd<true>(vk, ns, p, -c, gk);
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) {
                    aR.x[i] += gk.x[i];
                    if (tail_side) aH.x[i] += gk.x[i]; else aT.x[i] -= gk.x[i];
                    gs.x[i] = tail_side ? -gk.x[i] : gk.x[i];   // corrupted tail gets -g, corrupted head +g
                }
                if constexpr (MODEL == 0) {
                    if constexpr (CSR) {
                        if (!PT_ABLATE(P.dbg, 1)) vstore(gs, dst, D, lane);
                    } else {
                        sink.ent(e, gs, D, lane);
                    }
                } else {
                    Vec gp, ge;
                    if (nf) vnormalize_bwd<true>(Es, en, gs, gp); else gp = gs;
                    const float ng = vdot(nW, gp);
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) {
                        ge.x[i] = gp.x[i] - nW.x[i] * ng;
                        aW.x[i] -= ed * gp.x[i] + ng * E[k].x[i];
                    }
                    if constexpr (CSR) vstore(ge, dst, D, lane); else sink.ent(e, ge, D, lane);
                }
            }
        };
        if constexpr (DB) {
            for (int64_t c0 = k_lo; c0 < k_hi;) {
                if (c0 + NCH < k_hi) load_chunk(EB, c0 + NCH);
                process(EA, c0);
                c0 += NCH;
                if (c0 >= k_hi) break;
                if (c0 + NCH < k_hi) load_chunk(EA, c0 + NCH);
                process(EB, c0);
                c0 += NCH;
            }
        } else {
            for (int64_t c0 = k_lo; c0 < k_hi;) {
                process(EA, c0);
                c0 += NCH;
                if (c0 >= k_hi) break;
                load_chunk(EA, c0);
            }
        }
    }
    if constexpr (S > 1) {
        // ---- meet the positive's partials in LDS
        float *mr = red + grp * 4 * RW;
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) {
            const int c = ((k / VEC) * G + lane) * VEC + k % VEC;
            mr[0 * RW + c] = aH.x[k];
            mr[1 * RW + c] = aT.x[k];
            mr[2 * RW + c] = aR.x[k];
            if constexpr (MODEL == 1) mr[3 * RW + c] = aW.x[k];
        }
        if (lane == 0) {
            cs[grp * 2 + 0] = csum;
            cs[grp * 2 + 1] = lsum;
        }
        __syncthreads();
        if (sub != 0 || !active) return;
        csum = 0.f;
        lsum = 0.f;
        vzero(aH); vzero(aT); vzero(aR); vzero(aW);
        for (int q = 0; q < S; ++q) {   // fixed order: deterministic
            const float *qr = red + (grp + q) * 4 * RW;
#pragma unroll
            for (int k = 0; k < Vec::N; ++k) {
                const int c = ((k / VEC) * G + lane) * VEC + k % VEC;
                aH.x[k] += qr[0 * RW + c];
                aT.x[k] += qr[1 * RW + c];
                aR.x[k] += qr[2 * RW + c];
                if constexpr (MODEL == 1) aW.x[k] += qr[3 * RW + c];
            }
            csum += cs[(grp + q) * 2 + 0];
            lsum += cs[(grp + q) * 2 + 1];
        }
    }
    if (!active) return;
    // ---- positive backward and the group's on-chip accumulators
    if (uni<G>(csum) != 0.f) {
        Vec gv;
        vpnorm_bwd<true>(vpos, ps, p, csum, gv);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            aH.x[i] += gv.x[i];
            aR.x[i] += gv.x[i];
            aT.x[i] -= gv.x[i];
        }
        if constexpr (MODEL == 0) {
            if (!PT_ABLATE(P.dbg, 2)) {
                sink.rel(rp, aR, D, lane);
                sink.ent(hp, aH, D, lane);
                sink.ent(tp, aT, D, lane);
            }
        } else {
            sink.rel(rp, aR, D, lane);
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const Vec &acc = s2 == 0 ? aH : aT;
                const Vec &Ev = s2 == 0 ? H : T;
                const Vec &Esv = s2 == 0 ? Hs : Ts;
                const float enn = s2 == 0 ? hn : tn;
                const float edd = s2 == 0 ? hdot : tdot;
                Vec gp, ge;
                if (nf) vnormalize_bwd<true>(Esv, enn, acc, gp); else gp = acc;
                const float ng = vdot(nW, gp);
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) {
                    ge.x[i] = gp.x[i] - nW.x[i] * ng;
                    aW.x[i] -= edd * gp.x[i] + ng * Ev.x[i];
                }
                sink.ent(s2 == 0 ? hp : tp, ge, D, lane);
            }
            sink.norm(rp, aW, D, lane);
        }
    }
    if (lane == 0 && sink.lpart) sink.lpart[b] = lsum;
}

// Fused TransE step on a counting-sort batch (the C2 hot loop, CSR path). ONE lane group per positive
// takes all of its negatives: the positive's forward runs once (no sub-group split, no LDS meet), its
// negatives' records sit in registers (lane j of the group holds negative w0 + j of the current window
// of G) and are broadcast with readlane (G = 64: scalar entity ids, scalar branches) or a group
// shuffle; the rows of NCH negatives load while the previous NCH compute (double buffer).
// The kernel is VALU-issue bound at C2's shape, so the per-negative work is kept minimal: the tail-side
// base h-hat + r-hat is formed once (same association as (h + r) - t), the corrupted row's gradient is
// formed with the sign of its slot and stored to its counting-sort slot, and two accumulators collect
// the positive's rows: At = sum over tail-corrupted negatives of dL/dv, Ah over head-corrupted ones
// (dL/dh-hat = At + g+, dL/dr-hat = At + Ah + g+, dL/dt-hat = -(Ah + g+)).
template <int G>
__device__ __forceinline__ int32_t gbcast(int32_t v, int j) {
    if constexpr (G == 64) return __builtin_amdgcn_readlane(v, j); else return __shfl(v, j, G);
}

// SC: the slot-scale mode (CsrWork::slot_scale) as its own instantiation - its branches inside the default
// kernel had cost 1.5-2 us per C2 step (same-box A/B, tools_gpu/r05_ac.sh)
template <int G, int VEC, int KCH, int NCH, int S, int PN, int NT = 256, bool SC = false>
__global__ __launch_bounds__(NT) void k_step_csr(StepParams P, GlobalSink sink, CsrWork cw) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = NT / G;      // lane groups per block
    constexpr int PPB = GPB / S;     // positives per block
    constexpr int RW = KCH * G * VEC;
    __shared__ float red[S > 1 ? GPB * 2 * RW + 2 * GPB : 1];
    __shared__ float trb[PPB * 3 * RW];   // positive-row gradients, transposed for coalesced atomics
    const int lane = threadIdx.x % G;
    const int grp = threadIdx.x / G;
    const int sub = grp % S;
    const int64_t b = (int64_t)blockIdx.x * PPB + grp / S;
    const bool active = b < P.batch_size;   // group-uniform
    const int D = (int)P.dim;
    const uint32_t rowb = (uint32_t)D * 4u;
    const int neg = (int)P.neg;
    constexpr int p = PN;   // p_norm as a template parameter: no per-negative branch on it
    const bool nf = P.norm_flag != 0;
    const float m = P.margin, inv = P.inv_count;
    // sub-group `sub` takes negatives [k_lo, k_hi)
    const int nper = (neg + S - 1) / S;
    const int k_lo = sub * nper < neg ? sub * nper : neg;
    const int k_hi = k_lo + nper < neg ? k_lo + nper : neg;
    Vec At, Ah, rh, th, bt;   // (v+ = bt - th is re-formed where needed: fewer live registers)
    vzero(At); vzero(Ah); vzero(rh); vzero(th); vzero(bt);
    float csum = 0.f, lsum = 0.f, ps = 0.f;
    int32_t hp = 0, rp = 0, tp = 0;
    if (active) {
        const auto ent_rs = make_rsrc(P.ent, (uint32_t)P.ent_total * rowb);
        const auto rel_rs = make_rsrc(P.rel, (uint32_t)P.rel_total * rowb);
        const auto con_rs = make_rsrc(cw.contrib, (uint32_t)(P.batch_size * neg) * rowb);
        const int4 q = cw.pos[b];
        hp = uni<G>(q.x); rp = uni<G>(q.y); tp = uni<G>(q.z);
        const int32_t *nrec = cw.neg + b * neg;
        const int32_t *ndst = cw.off + b * neg;
        int w0 = k_lo, wend = k_hi - k_lo < G ? k_hi : k_lo + G;
        int32_t rec = 0, dst = 0;
        if (w0 + lane < wend) {
            rec = nrec[w0 + lane];
            dst = ndst[w0 + lane];
            if (cw.rank_only) dst += cw.start[rec >> 1];   // rank in the bucket -> destination row
        }
        Vec H, T, Rr;
        bload(H, ent_rs, (uint32_t)hp * rowb, D, lane);
        bload(T, ent_rs, (uint32_t)tp * rowb, D, lane);
        bload(Rr, rel_rs, (uint32_t)rp * rowb, D, lane);
        // every chunk issues exactly NCH row loads (past the window end: the window's last row again), so
        // the waits for a chunk never cover the next chunk's loads
        Vec EA[NCH], EB[NCH];
        auto load_chunk = [&](Vec(&E)[NCH], int k0) {
#pragma unroll
            for (int u = 0; u < NCH; ++u) {
                const int kk = k0 + u < wend ? k0 + u : wend - 1;
                const uint32_t e = (uint32_t)(gbcast<G>(rec, kk - w0) >> 1);
                bload(E[u], ent_rs, PT_ABLATE(P.dbg, 4) ? kOob : e * rowb, D, lane);
            }
        };
        if (w0 < wend) load_chunk(EA, w0);
        // ---- positive forward
        Vec hh, vpos;
        if (nf) {
            vnormalize<true>(H, hh);
            vnormalize<true>(Rr, rh);
            vnormalize<true>(T, th);
        } else {
            hh = H; rh = Rr; th = T;
        }
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            bt.x[i] = hh.x[i] + rh.x[i];
            vpos.x[i] = bt.x[i] - th.x[i];
        }
        ps = vpnorm<true>(vpos, p);
        constexpr bool scale_mode = SC;
        if (scale_mode && sub == 0) {   // the positive's normalized rows, for the apply pass to re-form slot rows
            const auto base_rs = make_rsrc(cw.bases, (uint32_t)(P.batch_size * 3) * rowb);
            bstore(bt, base_rs, (uint32_t)(b * 3) * rowb, D, lane);
            bstore(rh, base_rs, (uint32_t)(b * 3 + 1) * rowb, D, lane);
            bstore(th, base_rs, (uint32_t)(b * 3 + 2) * rowb, D, lane);
        }
        auto process = [&](Vec(&E)[NCH], int k0) {
#pragma unroll
            for (int u = 0; u < NCH; ++u) {
                if (k0 + u < wend) {   // (a guard, not a break: the loop must unroll fully, E[u] are registers)
                const int32_t r = gbcast<G>(rec, k0 + u - w0);
                const int32_t di = gbcast<G>(dst, k0 + u - w0);
                const uint32_t slot = (uint32_t)di * rowb;
                const bool tail_side = r & 1;
                Vec eh, vk, gs;
                if (nf) vnormalize<true>(E[u], eh); else eh = E[u];
                if constexpr (SC) {
#pragma clang fp contract(off)   // e-hat's product stays rounded: k_apply_buf's slot-scale mode re-forms v the same way
                    if (tail_side) {
#pragma unroll
                        for (int i = 0; i < Vec::N; ++i) vk.x[i] = bt.x[i] - eh.x[i];
                    } else {
#pragma unroll
                        for (int i = 0; i < Vec::N; ++i) vk.x[i] = (eh.x[i] + rh.x[i]) - th.x[i];
                    }
                } else {
                    if (tail_side) {
#pragma unroll
                        for (int i = 0; i < Vec::N; ++i) vk.x[i] = bt.x[i] - eh.x[i];
                    } else {
#pragma unroll
                        for (int i = 0; i < Vec::N; ++i) vk.x[i] = (eh.x[i] + rh.x[i]) - th.x[i];
                    }
                }
                const float ns = vpnorm<true>(vk, p);
                const float a = uni<G>(ps - ns);
                lsum += a > -m ? a : -m;
                const float c = a > -m ? inv : (a == -m ? inv * 0.5f : 0.f);
                csum += c;
                // slot gradient d loss / d e-hat: -g for a corrupted tail, +g for a corrupted head
                // (g = dL/dv); an inactive pair stores zeros (the reserved slot must be defined)
                vpnorm_bwd<true>(vk, ns, p, tail_side ? c : -c, gs);
                if constexpr (scale_mode) {
                    // the slot's record: its positive and side, and vpnorm_bwd's scalar (p = 2: ds / ns as the
                    // fast form computes it, p = 1: ds) - the apply pass forms gs again from them
                    const float ds = tail_side ? c : -c;
                    const float kk = p == 1 ? ds : (ns == 0.f ? 0.f : ds * frcp<true>(ns));
                    if (lane == 0) cw.srec[di] = make_int2((int32_t)(b << 1) | (tail_side ? 1 : 0), __float_as_int(kk));
                } else {
                    bstore(gs, con_rs, PT_ABLATE(P.dbg, 1) ? kOob : slot, D, lane);
                }
                if (tail_side) {
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) At.x[i] -= gs.x[i];
                } else {
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) Ah.x[i] += gs.x[i];
                }
                }
            }
        };
        while (w0 < wend) {
            for (int c0 = w0; c0 < wend;) {
                if (c0 + NCH < wend) load_chunk(EB, c0 + NCH);
                process(EA, c0);
                c0 += NCH;
                if (c0 >= wend) break;
                if (c0 + NCH < wend) load_chunk(EA, c0 + NCH);
                process(EB, c0);
                c0 += NCH;
            }
            w0 = wend;
            if (w0 >= k_hi) break;
            wend = k_hi - w0 < G ? k_hi : w0 + G;
            rec = dst = 0;
            if (w0 + lane < wend) {
                rec = nrec[w0 + lane];
                dst = ndst[w0 + lane];
                if (cw.rank_only) dst += cw.start[rec >> 1];
            }
            load_chunk(EA, w0);
        }
    }
    if constexpr (S > 1) {
        // ---- the sub-groups' partials meet in LDS; sub-group 0 sums them in a fixed order
        float *mr = red + grp * 2 * RW;
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) {
            const int c = ((k / VEC) * G + lane) * VEC + k % VEC;
            mr[c] = At.x[k];
            mr[RW + c] = Ah.x[k];
        }
        float *cs = red + GPB * 2 * RW;
        if (lane == 0) {
            cs[grp * 2 + 0] = csum;
            cs[grp * 2 + 1] = lsum;
        }
        __syncthreads();
        if (sub != 0 || !active) return;
        vzero(At); vzero(Ah);
        csum = lsum = 0.f;
        for (int q2 = 0; q2 < S; ++q2) {
            const float *qr = red + (grp + q2) * 2 * RW;
#pragma unroll
            for (int k = 0; k < Vec::N; ++k) {
                const int c = ((k / VEC) * G + lane) * VEC + k % VEC;
                At.x[k] += qr[c];
                Ah.x[k] += qr[RW + c];
            }
            csum += cs[(grp + q2) * 2 + 0];
            lsum += cs[(grp + q2) * 2 + 1];
        }
    }
    if (!active) return;
    if (lane == 0 && sink.lpart) sink.lpart[b] = lsum;
    if (uni<G>(csum) == 0.f || PT_ABLATE(P.dbg, 2)) return;   // no active pair: every accumulator is zero
    Vec gv, aH, aR, aT, vpos;
#pragma unroll
    for (int i = 0; i < Vec::N; ++i) vpos.x[i] = bt.x[i] - th.x[i];
    vpnorm_bwd<true>(vpos, ps, p, csum, gv);
#pragma unroll
    for (int i = 0; i < Vec::N; ++i) {
        aH.x[i] = At.x[i] + gv.x[i];
        aR.x[i] = (At.x[i] + Ah.x[i]) + gv.x[i];
        aT.x[i] = -(Ah.x[i] + gv.x[i]);
    }
    // float4 lanes make a row atomic touch 4x the cache lines per instruction: pass the three rows
    // through LDS so lane l adds floats l, l + G, ... (256 contiguous bytes per instruction at G = 64)
    float *tb = trb + (grp / S) * 3 * RW;
#pragma unroll
    for (int k = 0; k < Vec::N; ++k) {
        const int c = ((k / VEC) * G + lane) * VEC + k % VEC;
        tb[c] = aR.x[k];
        tb[RW + c] = aH.x[k];
        tb[2 * RW + c] = aT.x[k];
    }
    __builtin_amdgcn_wave_barrier();   // the group is within one wave: LDS order is program order
    float *gr = sink.grel + (int64_t)rp * D, *gh = sink.gent + (int64_t)hp * D, *gt = sink.gent + (int64_t)tp * D;
#pragma unroll
    for (int k = 0; k < KCH * VEC; ++k) {
        const int c = k * G + lane;
        if (c < D) {
            atomicAdd(gr + c, tb[c]);
            atomicAdd(gh + c, tb[RW + c]);
            atomicAdd(gt + c, tb[2 * RW + c]);
        }
    }
    if (lane == 0) {
        sink.frel[rp] = 1;
        sink.fent[hp] = 1;
        sink.fent[tp] = 1;
    }
}

}  // namespace dev

// ==================================================================== host launchers ===========
namespace {

// negatives held in registers per chunk: smallest of {1,4,8,32} >= neg, at most 128 VGPRs of rows
int pick_nch(int64_t neg, int kch) {
    static const int opts[4] = {1, 4, 8, 32};
    int best = 1;
    for (int o : opts) {
        if (o * kch > 128) break;
        best = o;
        if (o >= neg) break;
    }
    return best;
}

// VEC=1 shapes x NCH x S of the sampled step kernel: S = 1 for neg < 8 (NCH covers neg), S = 4 with
// NCH covering ceil(neg/4) (chunks beyond 32 negatives per sub-group loop)
#define PT_SSHAPES(X)                                                                                  \
    X(2, 1, 1, 1, 1, false) X(2, 1, 1, 4, 1, false) X(2, 1, 1, 8, 1, false) X(2, 1, 1, 8, 4, false) X(2, 1, 1, 32, 4, false)                  \
    X(4, 1, 1, 1, 1, false) X(4, 1, 1, 4, 1, false) X(4, 1, 1, 8, 1, false) X(4, 1, 1, 8, 4, false) X(4, 1, 1, 32, 4, false)                  \
    X(8, 1, 1, 1, 1, false) X(8, 1, 1, 4, 1, false) X(8, 1, 1, 8, 1, false) X(8, 1, 1, 8, 4, false) X(8, 1, 1, 32, 4, false)                  \
    X(16, 1, 1, 1, 1, false) X(16, 1, 1, 4, 1, false) X(16, 1, 1, 8, 1, false) X(16, 1, 1, 8, 4, false) X(16, 1, 1, 32, 4, false)             \
    X(32, 1, 1, 1, 1, false) X(32, 1, 1, 4, 1, false) X(32, 1, 1, 8, 1, false) X(32, 1, 1, 8, 4, false) X(32, 1, 1, 32, 4, false)             \
    X(64, 1, 1, 1, 1, false) X(64, 1, 1, 4, 1, false) X(64, 1, 1, 8, 1, false) X(64, 1, 1, 8, 4, false) X(64, 1, 1, 32, 4, false)             \
    X(64, 1, 2, 1, 1, false) X(64, 1, 2, 4, 1, false) X(64, 1, 2, 8, 1, false) X(64, 1, 2, 8, 4, false) X(64, 1, 2, 32, 4, false)             \
    X(64, 1, 4, 1, 1, false) X(64, 1, 4, 4, 1, false) X(64, 1, 4, 8, 1, false) X(64, 1, 4, 8, 4, false) X(64, 1, 4, 32, 4, false)             \
    X(64, 1, 4, 8, 2, false) X(64, 1, 4, 4, 4, false) X(64, 1, 4, 4, 2, false)                             \
    X(64, 1, 8, 1, 1, false) X(64, 1, 8, 4, 1, false) X(64, 1, 8, 8, 1, false) X(64, 1, 8, 8, 4, false)

}  // namespace
// k_step_csr instances (G, KCH, NCH), float4 lanes
#define PT_CSTEPS(X)                                                                                   \
    X(2, 1, 2, 1) X(4, 1, 2, 1) X(8, 1, 2, 1) X(16, 1, 2, 1) X(32, 1, 2, 1) X(64, 1, 2, 1)                \
    X(2, 1, 2, 2) X(4, 1, 2, 2) X(8, 1, 2, 2) X(16, 1, 2, 2) X(32, 1, 2, 2) X(64, 1, 2, 2)                \
    X(2, 1, 2, 4) X(4, 1, 2, 4) X(8, 1, 2, 4) X(16, 1, 2, 4) X(32, 1, 2, 4) X(64, 1, 2, 4)                \
    X(64, 1, 4, 4) X(64, 1, 1, 4) X(64, 2, 2, 1)             \
    X(64, 2, 2, 2) X(64, 2, 2, 4) X(64, 3, 2, 1) X(64, 3, 2, 4) X(64, 4, 2, 1) X(64, 4, 2, 4)

// TransE on the counting-sort path with float4 rows takes k_step_csr (PT_STEP_OLD=1: the sub-group
// kernel k_step_sampled); raw-buffer byte offsets must fit in 31 bits
static bool csr_fast_path(const StepParams &P) {
    static const bool old_step = [] {
        const char *v = pt_tuning_env("PT_STEP_OLD");
        return v && atoi(v) != 0;
    }();
    const int64_t lim = int64_t(1) << 31;
    const bool fits31 = (P.ent_total + P.rel_total + P.batch_size * P.neg) * P.dim * 4 < lim;
    return P.model == 0 && P.dim % 4 == 0 && fits31 && !old_step;
}

// whether launch_step can take this (P, neg) on the in-kernel-sampled path: k_step_csr has no LDS
// limit on neg; the sub-group kernel keeps a block's negative records in LDS (64 KB)
bool step_fits(const StepParams &P0, int64_t neg, bool csr) {
    StepParams P = P0;
    P.neg = neg;
    if (csr && csr_fast_path(P)) return true;
    const Shape s = pick_shape(P.dim, false);
    const int S = (neg >= 8 && 256 / s.G >= 4) ? 4 : 1;
    const int64_t gpb = 256 / s.G, ppb = gpb / S;
    size_t lds = (size_t)ppb * (size_t)neg * sizeof(int64_t) * (csr ? 2 : 1);
    if (S > 1) lds += sizeof(float) * ((size_t)gpb * 4 * s.KCH * s.G * s.VEC + (size_t)gpb * 2);
    return lds <= 64 * 1024;
}

hipError_t launch_step(const StepParams &P, const DeviceGraph &g, const uint64_t *states, int64_t threads, int bern,
                       int filter, const int64_t *bh, const int64_t *bt, const int64_t *br, const StepWorkspace &W,
                       float *loss, hipStream_t st, const CsrWork *csr) {
    if (P.batch_size <= 0) return hipSuccess;
    dev::GlobalSink sink{W.gent, W.grel, W.gnorm, W.fent, W.frel, W.fnorm, W.lpart};
    if (bh) {   // external batch
        const Shape s = pick_shape(P.dim);
        const int64_t gpb = 256 / s.G;
        const dim3 grid((unsigned)((P.batch_size + gpb - 1) / gpb)), block(256);
#define PT_STEP(G_, V_, K_)                                                                                        \
        if (s.G == G_ && s.VEC == V_ && s.KCH == K_) {                                                           \
            if (P.model == 0)                                                                                      \
                hipLaunchKernelGGL((dev::k_step<0, G_, V_, K_>), grid, block, 0, st, P, bh, bt, br, sink, loss);   \
            else                                                                                                   \
                hipLaunchKernelGGL((dev::k_step<1, G_, V_, K_>), grid, block, 0, st, P, bh, bt, br, sink, loss);   \
            return hipGetLastError();                                                                              \
        }
        PT_SHAPES(PT_STEP)
#undef PT_STEP
        return hipErrorInvalidValue;
    }
    // TransE on a counting-sort batch with float4 rows: k_step_csr (S lane groups per positive);
    // PT_STEP_G / PT_STEP_S / PT_STEP_NCH override its shape
    if (csr && csr_fast_path(P)) {
        const int64_t chunks = P.dim / 4;
        int G = 2;
        while (G < chunks && G < 64) G <<= 1;
        if (const char *v = pt_tuning_env("PT_STEP_G")) G = atoi(v);
        const int KCH = (int)((chunks + G - 1) / G);
        // split a positive's negatives over S lane groups of one block (more waves in flight: the step
        // is latency-bound when one group walks all negatives)
        int S = 1;
        while (S < 4 && S * 2 <= 256 / G && P.neg >= 6 * S * 2) S *= 2;
        if (const char *v = pt_tuning_env("PT_STEP_S")) S = atoi(v);
        int nch = 2;   // C2 (S = 4, 7 negatives per group): chunks of 2 rows, double-buffered, measured fastest
        if (const char *v = pt_tuning_env("PT_STEP_NCH")) nch = atoi(v);
#define PT_CSTEP(G_, K_, N_, S_)                                                                       \
        if (G == G_ && KCH == K_ && nch == N_ && S == S_) {                                          \
            constexpr int NT_ = S_ * G_ >= 256 || 256 % (S_ * G_) != 0 ? S_ * G_ : 256;             \
            const dim3 grid((unsigned)((P.batch_size * S_ * G_ + NT_ - 1) / NT_)), block(NT_);        \
            if (csr->slot_scale && P.p_norm == 1)                                                    \
                hipLaunchKernelGGL((dev::k_step_csr<G_, 4, K_, N_, S_, 1, NT_, true>), grid, block, 0, st, P, sink, *csr); \
            else if (csr->slot_scale)                                                                \
                hipLaunchKernelGGL((dev::k_step_csr<G_, 4, K_, N_, S_, 2, NT_, true>), grid, block, 0, st, P, sink, *csr); \
            else if (P.p_norm == 1)                                                                  \
                hipLaunchKernelGGL((dev::k_step_csr<G_, 4, K_, N_, S_, 1, NT_>), grid, block, 0, st, P, sink, *csr); \
            else                                                                                     \
                hipLaunchKernelGGL((dev::k_step_csr<G_, 4, K_, N_, S_, 2, NT_>), grid, block, 0, st, P, sink, *csr); \
            return hipGetLastError();                                                                \
        }
        PT_CSTEPS(PT_CSTEP)
#undef PT_CSTEP
    }
    // row layout: one float per lane (each wave instruction moves 64 contiguous floats)
    {
        const Shape s = pick_shape(P.dim, false);
        // split a positive's negatives over 4 lane groups when there are enough of them
        // (PT_STEP_S = 1 | 2 | 4 and PT_STEP_NCH override, for tuning)
        int S = (P.neg >= 8 && 256 / s.G >= 4) ? 4 : 1;
        if (const char *v = pt_tuning_env("PT_STEP_S")) {
            const int want = atoi(v);
            if ((want == 1 || want == 2 || want == 4) && 256 / s.G >= want) S = want;
        }
        const int64_t nper = (P.neg + S - 1) / S;
        int nch = pick_nch(nper, s.KCH * s.VEC);
        if (const char *v = pt_tuning_env("PT_STEP_NCH")) nch = atoi(v);
        // double-buffer the negative rows when a lane group takes more than one chunk (PT_STEP_DB=0 off)
        bool db = nper > nch;
        if (const char *v = pt_tuning_env("PT_STEP_DB")) db = db && atoi(v) != 0;
        const int64_t gpb = 256 / s.G, ppb = gpb / S;
        const dim3 grid((unsigned)((P.batch_size + ppb - 1) / ppb)), block(256);
        size_t lds = (size_t)ppb * (size_t)P.neg * sizeof(int64_t) * (csr ? 2 : 1);
        if (S > 1) lds += sizeof(float) * ((size_t)gpb * 4 * s.KCH * s.G * s.VEC + (size_t)gpb * 2);
        if (lds > 64 * 1024) return hipErrorInvalidValue;
        const CsrWork cw = csr ? *csr : CsrWork{};
#define PT_SSTEP(G_, V_, K_, N_, S_, DB_)                                                                            \
        if (s.G == G_ && s.VEC == V_ && s.KCH == K_ && nch == N_ && S == S_ && db == DB_) {                              \
            if (csr) {                                                                                            \
                if (P.model == 0)                                                                                 \
                    hipLaunchKernelGGL((dev::k_step_sampled<0, G_, V_, K_, N_, S_, true, DB_>), grid, block, lds, st,   \
                                       P, g, states, threads, bern, filter, sink, loss, cw);                      \
                else                                                                                              \
                    hipLaunchKernelGGL((dev::k_step_sampled<1, G_, V_, K_, N_, S_, true, DB_>), grid, block, lds, st,   \
                                       P, g, states, threads, bern, filter, sink, loss, cw);                      \
            } else {                                                                                              \
                if (P.model == 0)                                                                                 \
                    hipLaunchKernelGGL((dev::k_step_sampled<0, G_, V_, K_, N_, S_, false, DB_>), grid, block, lds, st,  \
                                       P, g, states, threads, bern, filter, sink, loss, cw);                      \
                else                                                                                              \
                    hipLaunchKernelGGL((dev::k_step_sampled<1, G_, V_, K_, N_, S_, false, DB_>), grid, block, lds, st,  \
                                       P, g, states, threads, bern, filter, sink, loss, cw);                      \
            }                                                                                                     \
            return hipGetLastError();                                                                             \
        }
        // the preferred chunk size first, then any instantiated one (the kernel loops over chunks);
        // double-buffered instances are tuning experiments only
        const int cands[6] = {nch, nch, 8, 4, 32, 1};
        for (int ci = 0; ci < 6; ++ci) {
            nch = cands[ci];
            if (ci > 0) db = false;
            PT_SSHAPES(PT_SSTEP)
        }
#undef PT_SSTEP
    }
    return hipErrorInvalidValue;
}

}  // namespace pt
