// HIP kernels of the PuTransE / TransE / TransH hot path for gfx950 (MI355X).
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

#include "device.h"
#include "graph.h"
#include "kernels.h"
#include "rng.h"

namespace pt {
namespace dev {

// sampling() into arrays (one thread per positive); the stream advance is a separate kernel
__global__ void k_sample(DeviceGraph g, const uint64_t *__restrict__ states, int64_t threads, int64_t bs, int64_t neg,
                         int bern, int filter, int64_t *__restrict__ oh, int64_t *__restrict__ ot,
                         int64_t *__restrict__ orr, float *__restrict__ oy) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= bs) return;
    const PosDraw pd = draw_positive(g, states, threads, bs, b, 1 + 2 * neg);
    const int64_t hp = pd.h, rp = pd.r, tp = pd.t;
    oh[b] = hp; ot[b] = tp; orr[b] = rp;
    if (oy) oy[b] = 1.f;
    for (int64_t k = 0; k < neg; ++k) {
        int tail_side;
        const int64_t e = draw_negative(g, pd, k, bern, filter, &tail_side);
        const int64_t o = (k + 1) * bs + b;
        oh[o] = tail_side ? hp : e;
        ot[o] = tail_side ? e : tp;
        orr[o] = rp;
        if (oy) oy[o] = -1.f;
    }
}

// busy-waits `us` microseconds (100 MHz constant wall clock): keeps a stream occupied while the host
// enqueues a measured sequence behind it
__global__ void k_spin(int64_t us) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < (uint64_t)us * 100) __builtin_amdgcn_s_sleep(8);
}

__global__ void k_advance(uint64_t *states, int64_t threads, int64_t bs, int64_t dpp) {
    advance_states(states, threads, bs, dpp, (int)threadIdx.x);
}

// Counting-sort (CSR) sampling pass of the large-negative path: one thread per (positive, negative)
// slot draws exactly what getBatch draws for it (stream jump to the slot) and reserves the slot's
// place in its corrupted entity's bucket. Thread k == neg of a positive records the positive.
using pt::CsrWork;

__global__ __launch_bounds__(256) void k_sample_csr(DeviceGraph g, const uint64_t *__restrict__ states,
                                                    int64_t threads, int64_t bs, int64_t neg, int bern, int filter,
                                                    int64_t calls, CsrWork w) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_call = bs * (neg + 1);
    if (idx >= calls * per_call) return;
    const int64_t call = idx / per_call, rem = idx - call * per_call;
    const int64_t b = rem / (neg + 1), k = rem - b * (neg + 1);
    const PosDraw pd = draw_positive(g, states, threads, bs, b, 1 + 2 * neg, call);
    if (k == neg) {
        w.pos[call * bs + b] = make_int4((int)pd.h, (int)pd.r, (int)pd.t, 0);
        return;
    }
    int side;
    const int64_t e = draw_negative(g, pd, k, bern, filter, &side);
    const int64_t o = call * bs * neg + b * neg + k;
    w.neg[o] = (int32_t)((e << 1) | side);
    w.off[o] = atomicAdd(&w.cnt[call * w.cnt_stride + e], 1);
}

// exclusive scan of the bucket sizes (one workgroup of 1024 threads, tiles of 16384 counts: 16
// contiguous counts per thread, wave shuffles for the thread totals, LDS for the 16 wave totals),
// zeroing the counts for the next step; also advances the sampler streams by this call's draws
// (the sampling pass was their only reader)
__global__ __launch_bounds__(1024) void k_scan_counts(int32_t *__restrict__ cnt_all, int32_t *__restrict__ start_all,
                                                      int64_t n, uint64_t *states, int64_t threads, int64_t bs,
                                                      int64_t dpp, CsrWork w, int64_t slots) {
    __shared__ int32_t wtot[16];
    __shared__ int32_t carry_s;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // one workgroup per sampled call; workgroup 0 advances the streams by all the calls' draws
    int32_t *cnt = cnt_all + (int64_t)blockIdx.x * ((n + 3) & ~int64_t(3));        // rows padded to 16 B
    int32_t *start = start_all + (int64_t)blockIdx.x * ((n + 4) & ~int64_t(3));
    if (blockIdx.x == 0 && tid < 64 && states) advance_states(states, threads, bs, dpp * (int64_t)gridDim.x, tid);
    if (tid == 0) carry_s = 0;
    __syncthreads();
    for (int64_t base = 0; base < n; base += 16384) {
        const int64_t lo = base + (int64_t)tid * 16;
        int32_t v[16];
        if (lo + 16 <= n) {
            const int4 *p4 = reinterpret_cast<const int4 *>(cnt + lo);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int4 x = p4[q];
                v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = lo + q < n ? cnt[lo + q] : 0;
        }
        int32_t tsum = 0;
#pragma unroll
        for (int q = 0; q < 16; ++q) tsum += v[q];
        int32_t incl = tsum;   // inclusive wave scan of the thread totals
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wtot[wid] = incl;
        __syncthreads();
        int32_t wpre = 0, total = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const int32_t t = wtot[w];
            wpre += w < wid ? t : 0;
            total += t;
        }
        int32_t run = carry_s + wpre + incl - tsum;
        if (lo + 16 <= n) {
            int32_t o[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                o[q] = run;
                run += v[q];
            }
            int4 *s4 = reinterpret_cast<int4 *>(start + lo);
            int4 *c4 = reinterpret_cast<int4 *>(cnt + lo);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                s4[q] = make_int4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
                c4[q] = make_int4(0, 0, 0, 0);
            }
        } else {
            for (int q = 0; q < 16 && lo + q < n; ++q) {
                start[lo + q] = run;
                run += v[q];
                cnt[lo + q] = 0;
            }
        }
        __syncthreads();
        if (tid == 0) carry_s += total;
        __syncthreads();
    }
    if (tid == 0) start[n] = carry_s;
    __syncthreads();
    // resolve every slot's destination row in the contribution buffer: start[e] + rank (the step kernel
    // then needs no dependent lookup). off[] is overwritten in place by the destination.
    const int32_t *neg = w.neg + (int64_t)blockIdx.x * slots;
    int32_t *off = w.off + (int64_t)blockIdx.x * slots;
    for (int64_t i = tid; i < slots; i += 1024) off[i] = start[neg[i] >> 1] + off[i];
}

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
                s_dst[pl * neg + k] = cw.off[b * neg + k];   // resolved destination (k_scan_counts)
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
                if (c0 + k < k_hi && !(P.dbg & 4)) vload(E[k], P.ent + (mine[c0 + k] >> 1) * D, D, lane);
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
                        if (!(P.dbg & 1)) vstore(gs, dst, D, lane);
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
            if (!(P.dbg & 2)) {
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

template <int G, int VEC, int KCH, int NCH, int S, int PN>
__global__ __launch_bounds__(256) void k_step_csr(StepParams P, GlobalSink sink, CsrWork cw) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;     // lane groups per block
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
    Vec At, Ah, vpos;
    vzero(At); vzero(Ah); vzero(vpos);
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
                bload(E[u], ent_rs, e * rowb, D, lane);
            }
        };
        if (w0 < wend) load_chunk(EA, w0);
        // ---- positive forward
        Vec hh, rh, th, bt;
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
        auto process = [&](Vec(&E)[NCH], int k0) {
#pragma unroll
            for (int u = 0; u < NCH; ++u) {
                if (k0 + u < wend) {   // (a guard, not a break: the loop must unroll fully, E[u] are registers)
                const int32_t r = gbcast<G>(rec, k0 + u - w0);
                const uint32_t slot = (uint32_t)gbcast<G>(dst, k0 + u - w0) * rowb;
                const bool tail_side = r & 1;
                Vec eh, vk, gs;
                if (nf) vnormalize<true>(E[u], eh); else eh = E[u];
                if (tail_side) {
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) vk.x[i] = bt.x[i] - eh.x[i];
                } else {
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) vk.x[i] = (eh.x[i] + rh.x[i]) - th.x[i];
                }
                const float ns = vpnorm<true>(vk, p);
                const float a = uni<G>(ps - ns);
                lsum += a > -m ? a : -m;
                const float c = a > -m ? inv : (a == -m ? inv * 0.5f : 0.f);
                csum += c;
                // slot gradient d loss / d e-hat: -g for a corrupted tail, +g for a corrupted head
                // (g = dL/dv); an inactive pair stores zeros (the reserved slot must be defined)
                vpnorm_bwd<true>(vk, ns, p, tail_side ? c : -c, gs);
                bstore(gs, con_rs, slot, D, lane);
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
    if (uni<G>(csum) == 0.f) return;   // no active pair: every accumulator is zero
    Vec gv, aH, aR, aT;
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
        if (lane == 0) *A.loss += s * A.inv_count + A.margin;
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

// ---------------------------------------------------------------- scoring ----------------------
// model.predict over n triples (mode 0 normal, 1 head_batch: h varies, 2 tail_batch: t varies)
template <int MODEL, int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_score(StepParams P, int mode, const int64_t *__restrict__ h,
                                               const int64_t *__restrict__ t, const int64_t *__restrict__ r,
                                               int64_t n, float *__restrict__ out) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    const int lane = threadIdx.x % G;
    const int64_t i = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    if (i >= n) return;
    const int D = (int)P.dim;
    const int64_t hi = h[mode == 1 || mode == 0 ? i : 0];
    const int64_t ti = t[mode == 2 || mode == 0 ? i : 0];
    const int64_t ri = r[mode == 0 ? i : 0];
    Vec H, T, R, hh, th, rh, v;
    vload(H, P.ent + hi * D, D, lane);
    vload(T, P.ent + ti * D, D, lane);
    vload(R, P.rel + ri * D, D, lane);
    if constexpr (MODEL == 1) {
        Vec W, nW;
        vload(W, P.normv + ri * D, D, lane);
        vnormalize(W, nW);
        const float hd = vdot(H, nW), td = vdot(T, nW);
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) {
            H.x[k] = H.x[k] - hd * nW.x[k];
            T.x[k] = T.x[k] - td * nW.x[k];
        }
    }
    if (P.norm_flag) {
        vnormalize(H, hh);
        vnormalize(R, rh);
        vnormalize(T, th);
    } else {
        hh = H; rh = R; th = T;
    }
#pragma unroll
    for (int k = 0; k < Vec::N; ++k)
        v.x[k] = mode == 1 ? hh.x[k] + (rh.x[k] - th.x[k]) : (hh.x[k] + rh.x[k]) - th.x[k];
    const float s = vpnorm(v, P.p_norm);
    if (lane == 0) out[i] = s;
}

// Candidate scoring for link prediction: row q holds the scores of query q's candidate list in the
// order getHeadBatch/getTailBatch emit it ([truth, 0..E-1 without truth], Test.h:37-107), with the
// association of model.predict for that mode (head_batch: h + (r - t); tail_batch: (h + r) - t).
template <int MODEL, int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_score_queries(StepParams P, int side, const int64_t *__restrict__ qh,
                                                       const int64_t *__restrict__ qt, const int64_t *__restrict__ qr,
                                                       int64_t nq, int64_t E, float *__restrict__ out, int global_order) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    const int lane = threadIdx.x % G;
    const int grp = threadIdx.x / G;
    const int64_t q = blockIdx.y;
    if (q >= nq) return;
    const int D = (int)P.dim;
    const int64_t h = qh[q], t = qt[q], r = qr[q];
    const int64_t truth = side == 0 ? h : t;
    const int64_t anchor = side == 0 ? t : h;
    Vec A, R, ah, rh, nW, base;
    vload(A, P.ent + anchor * D, D, lane);
    vload(R, P.rel + r * D, D, lane);
    if constexpr (MODEL == 1) {
        Vec W;
        vload(W, P.normv + r * D, D, lane);
        vnormalize(W, nW);
        const float ad = vdot(A, nW);
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) A.x[k] = A.x[k] - ad * nW.x[k];
    }
    if (P.norm_flag) {
        vnormalize(A, ah);
        vnormalize(R, rh);
    } else {
        ah = A; rh = R;
    }
#pragma unroll
    for (int k = 0; k < Vec::N; ++k) base.x[k] = side == 0 ? rh.x[k] - ah.x[k] : ah.x[k] + rh.x[k];
    float *row = out + q * E;
    for (int64_t j = (int64_t)blockIdx.x * GPB + grp; j < E; j += (int64_t)gridDim.x * GPB) {
        // candidate order of getHeadBatch/getTailBatch ([truth, 0..E-1 without truth], Test.h:37-107),
        // or column = entity id (global_order, the layout pt_rank_rows ranks)
        const int64_t e = global_order ? j : (j == 0 ? truth : (j - 1 < truth ? j - 1 : j));
        Vec X, xh, v;
        vload(X, P.ent + e * D, D, lane);
        if constexpr (MODEL == 1) {
            const float xd = vdot(X, nW);
#pragma unroll
            for (int k = 0; k < Vec::N; ++k) X.x[k] = X.x[k] - xd * nW.x[k];
        }
        if (P.norm_flag) vnormalize(X, xh); else xh = X;
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) v.x[k] = side == 0 ? xh.x[k] + base.x[k] : base.x[k] - xh.x[k];
        const float s = vpnorm(v, P.p_norm);
        if (lane == 0) row[j] = s;
    }
}

// ---------------------------------------------------------------- universe link prediction ------
// Global energy estimation (Parallel_Universe_Config.py:446-554): for every (key, universe) pair score
// every local entity of the universe as the missing side and MIN it into the key's global row
// (scores are norms >= 0, so float order == int order and atomicMin on the bits is exact).
// side 0 = head prediction (anchor is the tail: e + (r - anchor)), side 1 = tail prediction
// (anchor is the head: (anchor + r) - e).
//
// k_lp_bases: one lane group per pair: the pair's normalized (projected for TransH) anchor combined
//   with its relation -> base[pair][D] (+ the relation's normal for TransH), and the null_vector tuple
//   score of the key in this universe (calc_tuple_score, :378-388: raw anchor, no projection).
// k_lp_scan: one workgroup per (entity chunk, universe): each entity row is loaded (and, for TransE,
//   normalized) ONCE and scored against every pair of its universe - the universe's rows are read once
//   per chunk instead of once per pair.
template <int MODEL, int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_lp_bases(const LpUniverseDev *__restrict__ us, const LpPair *__restrict__ pairs,
                                                  int64_t n_pairs, int p_norm, int norm_flag, float *__restrict__ base,
                                                  float *__restrict__ normal, float *__restrict__ tuple_min) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    const int lane = threadIdx.x % G;
    const int64_t pi = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    if (pi >= n_pairs) return;
    const LpPair pr = pairs[pi];
    const LpUniverseDev U = us[pr.universe];
    const int D = (int)U.dim;
    Vec A, R, ah, rh, nW, b;
    vload(A, U.ent + (int64_t)pr.anchor * D, D, lane);
    vload(R, U.rel + (int64_t)pr.rel * D, D, lane);
    if (norm_flag) vnormalize(R, rh); else rh = R;
    if (tuple_min) {
        Vec an, v;
        if (norm_flag) vnormalize(A, an); else an = A;
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) v.x[k] = pr.side == 0 ? rh.x[k] - an.x[k] : an.x[k] + rh.x[k];
        const float sc = vpnorm(v, p_norm);
        if (lane == 0) atomicMin(reinterpret_cast<int *>(tuple_min + pr.key), __float_as_int(sc));
    }
    if constexpr (MODEL == 1) {
        Vec W;
        vload(W, U.normv + (int64_t)pr.rel * D, D, lane);
        vnormalize(W, nW);
        const float ad = vdot(A, nW);
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) A.x[k] = A.x[k] - ad * nW.x[k];
        vstore(nW, normal + pi * D, D, lane);
    }
    if (norm_flag) vnormalize(A, ah); else ah = A;
#pragma unroll
    for (int k = 0; k < Vec::N; ++k) b.x[k] = pr.side == 0 ? rh.x[k] - ah.x[k] : ah.x[k] + rh.x[k];
    vstore(b, base + pi * D, D, lane);
}

template <int MODEL, int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_lp_scan(const LpUniverseDev *__restrict__ us, const LpPair *__restrict__ pairs,
                                                 const int64_t *__restrict__ uoff, const int32_t *__restrict__ uids,
                                                 int p_norm, int norm_flag, int64_t global_E,
                                                 const float *__restrict__ base, const float *__restrict__ normal,
                                                 float *__restrict__ rows) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    constexpr int EPG = 4;   // entities per lane group: each pair's base row is loaded once per 4 entities
    const int lane = threadIdx.x % G;
    const int grp = threadIdx.x / G;
    const int32_t u = uids[blockIdx.y];
    const LpUniverseDev U = us[u];
    const int D = (int)U.dim;
    const int64_t p0 = uoff[2 * u], p1 = uoff[2 * u + 1];   // the universe's pairs (relative to `pairs`)
    const int64_t stride = (int64_t)gridDim.x * GPB * EPG;
    for (int64_t e0 = ((int64_t)blockIdx.x * GPB + grp) * EPG; e0 < U.ent_total; e0 += stride) {
        Vec X[EPG], xh[EPG];
        int64_t col[EPG];
#pragma unroll
        for (int q = 0; q < EPG; ++q) {
            const int64_t e = e0 + q < U.ent_total ? e0 + q : U.ent_total - 1;   // tail: repeat the last row
            vload(X[q], U.ent + e * D, D, lane);
            col[q] = e0 + q < U.ent_total ? U.remap[e] : -1;
        }
        if constexpr (MODEL == 0) {
#pragma unroll
            for (int q = 0; q < EPG; ++q) {
                if (norm_flag) vnormalize(X[q], xh[q]); else xh[q] = X[q];
            }
        }
        for (int64_t pi = p0; pi < p1; ++pi) {
            const LpPair pr = pairs[pi];
            Vec b;
            vload(b, base + pi * D, D, lane);
            Vec nW;
            if constexpr (MODEL == 1) vload(nW, normal + pi * D, D, lane);
#pragma unroll
            for (int q = 0; q < EPG; ++q) {
                if constexpr (MODEL == 1) {
                    Vec xp;
                    const float xd = vdot(X[q], nW);
#pragma unroll
                    for (int k = 0; k < Vec::N; ++k) xp.x[k] = X[q].x[k] - xd * nW.x[k];
                    if (norm_flag) vnormalize(xp, xh[q]); else xh[q] = xp;
                }
                Vec v;
#pragma unroll
                for (int k = 0; k < Vec::N; ++k) v.x[k] = pr.side == 0 ? xh[q].x[k] + b.x[k] : b.x[k] - xh[q].x[k];
                const float sc = vpnorm(v, p_norm);
                if (lane == 0 && col[q] >= 0)
                    atomicMin(reinterpret_cast<int *>(rows + (int64_t)pr.key * global_E + col[q]), __float_as_int(sc));
            }
        }
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
    X(64, 1, 4, 8, 1, true) X(64, 1, 4, 8, 2, true) X(64, 1, 4, 4, 1, true) X(64, 1, 4, 4, 2, true)         \
    X(64, 1, 4, 4, 4, true)                                                                                \
    X(64, 1, 8, 1, 1, false) X(64, 1, 8, 4, 1, false) X(64, 1, 8, 8, 1, false) X(64, 1, 8, 8, 4, false)                                \
    X(8, 4, 1, 1, 1, false) X(8, 4, 1, 4, 1, false) X(8, 4, 1, 8, 1, false) X(8, 4, 1, 8, 4, false)                                    \
    X(16, 4, 1, 1, 1, false) X(16, 4, 1, 4, 1, false) X(16, 4, 1, 8, 1, false) X(16, 4, 1, 8, 4, false)                                \
    X(32, 4, 1, 1, 1, false) X(32, 4, 1, 4, 1, false) X(32, 4, 1, 8, 1, false) X(32, 4, 1, 8, 4, false)                                \
    X(64, 4, 1, 1, 1, false) X(64, 4, 1, 4, 1, false) X(64, 4, 1, 8, 1, false) X(64, 4, 1, 8, 4, false) X(64, 4, 1, 32, 4, false)             \
    X(64, 4, 2, 1, 1, false) X(64, 4, 2, 4, 1, false) X(64, 4, 2, 8, 1, false) X(64, 4, 2, 8, 4, false)

}  // namespace

bool shape_supported(int64_t dim) {
    if (dim <= 0) return false;
    bool a = false, b = false;
    const Shape s = pick_shape(dim), s1 = pick_shape(dim, false);
#define PT_SUP(g, v, k) if (s.G == g && s.VEC == v && s.KCH == k) a = true; \
                        if (s1.G == g && s1.VEC == v && s1.KCH == k) b = true;
    PT_SHAPES(PT_SUP)
#undef PT_SUP
    return a && b;
}

// k_step_csr instances (G, KCH, NCH), float4 lanes
#define PT_CSTEPS(X)                                                                                   \
    X(2, 1, 8, 1) X(4, 1, 8, 1) X(8, 1, 8, 1) X(16, 1, 8, 1) X(32, 1, 8, 1) X(64, 1, 8, 1)                \
    X(2, 1, 4, 1) X(4, 1, 4, 1) X(8, 1, 4, 1) X(16, 1, 4, 1) X(32, 1, 4, 1) X(64, 1, 4, 1)                \
    X(4, 1, 8, 2) X(8, 1, 8, 2) X(16, 1, 8, 2) X(32, 1, 8, 2) X(64, 1, 8, 2)                             \
    X(4, 1, 8, 4) X(8, 1, 8, 4) X(16, 1, 8, 4) X(32, 1, 8, 4) X(64, 1, 8, 4)                             \
    X(4, 1, 4, 4) X(8, 1, 4, 4) X(16, 1, 4, 4) X(32, 1, 4, 4) X(64, 1, 4, 4)                             \
    X(64, 2, 4, 1) X(64, 2, 4, 2) X(64, 2, 4, 4) X(64, 3, 4, 1) X(64, 3, 4, 4) X(64, 4, 4, 1) X(64, 4, 4, 4)

hipError_t launch_sample(const DeviceGraph &g, const uint64_t *states, int64_t threads, int64_t bs, int64_t neg,
                         int bern, int filter, int64_t *h, int64_t *t, int64_t *r, float *y, hipStream_t st) {
    if (bs <= 0) return hipSuccess;
    const int bl = 256;
    hipLaunchKernelGGL(dev::k_sample, dim3((unsigned)((bs + bl - 1) / bl)), dim3(bl), 0, st, g, states, threads, bs,
                       neg, bern, filter, h, t, r, y);
    return hipGetLastError();
}

hipError_t launch_spin(int64_t us, hipStream_t st) {
    hipLaunchKernelGGL(dev::k_spin, dim3(1), dim3(64), 0, st, us);
    return hipGetLastError();
}

hipError_t launch_advance(uint64_t *states, int64_t threads, int64_t bs, int64_t dpp, hipStream_t st) {
    hipLaunchKernelGGL(dev::k_advance, dim3(1), dim3(64), 0, st, states, threads, bs, dpp);
    return hipGetLastError();
}

hipError_t launch_sample_csr(const DeviceGraph &g, const uint64_t *states, int64_t threads, int64_t bs, int64_t neg,
                             int bern, int filter, int64_t calls, const CsrWork &w, hipStream_t st) {
    const int64_t n = calls * bs * (neg + 1);
    hipLaunchKernelGGL(dev::k_sample_csr, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, states, threads, bs,
                       neg, bern, filter, calls, w);
    return hipGetLastError();
}

hipError_t launch_scan_counts(const CsrWork &w, int64_t n, int64_t calls, uint64_t *states, int64_t threads,
                              int64_t bs, int64_t dpp, hipStream_t st) {
    hipLaunchKernelGGL(dev::k_scan_counts, dim3((unsigned)calls), dim3(1024), 0, st, w.cnt, w.start, n, states, threads,
                       bs, dpp, w, bs * ((dpp - 1) / 2));
    return hipGetLastError();
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
    // TransE on a counting-sort batch with float4 rows: one lane group per positive (k_step_csr);
    // PT_STEP_OLD=1 keeps the sub-group kernel below, PT_STEP_G / PT_STEP_NCH pick the shape
    static const bool old_step = [] {
        const char *v = getenv("PT_STEP_OLD");
        return v && atoi(v) != 0;
    }();
    // (raw-buffer offsets must fit in 31 bits)
    const int64_t lim = int64_t(1) << 31;
    const bool fits31 = (P.ent_total + P.rel_total + P.batch_size * P.neg) * P.dim * 4 < lim;
    if (csr && P.model == 0 && P.dim % 4 == 0 && fits31 && !old_step) {
        const int64_t chunks = P.dim / 4;
        int G = 2;
        while (G < chunks && G < 64) G <<= 1;
        if (const char *v = getenv("PT_STEP_G")) G = atoi(v);
        const int KCH = (int)((chunks + G - 1) / G);
        // split a positive's negatives over S lane groups of one block (more waves in flight: the step
        // is latency-bound when one group walks all negatives)
        int S = 1;
        while (S < 4 && S * 2 <= 256 / G && P.neg >= 6 * S * 2) S *= 2;
        if (const char *v = getenv("PT_STEP_S")) S = atoi(v);
        const int64_t nper = (P.neg + S - 1) / S;
        int nch = KCH == 1 ? 8 : 4;
        if (nper <= 4 && KCH == 1) nch = 4;
        if (const char *v = getenv("PT_STEP_NCH")) nch = atoi(v);
        const int64_t ppb = 256 / G / S;
        const dim3 grid((unsigned)((P.batch_size + ppb - 1) / ppb)), block(256);
#define PT_CSTEP(G_, K_, N_, S_)                                                                       \
        if (G == G_ && KCH == K_ && nch == N_ && S == S_) {                                          \
            if (P.p_norm == 1)                                                                       \
                hipLaunchKernelGGL((dev::k_step_csr<G_, 4, K_, N_, S_, 1>), grid, block, 0, st, P, sink, *csr); \
            else                                                                                     \
                hipLaunchKernelGGL((dev::k_step_csr<G_, 4, K_, N_, S_, 2>), grid, block, 0, st, P, sink, *csr); \
            return hipGetLastError();                                                                \
        }
        PT_CSTEPS(PT_CSTEP)
#undef PT_CSTEP
    }
    // row layout: one float per lane (each wave instruction moves 64 contiguous floats), or float4
    // lanes when PT_STEP_VEC=4 and D % 4 == 0 (measured slower on the C2 step: 48.9 vs 40.6 us)
    const char *vec_env = getenv("PT_STEP_VEC");
    const bool try_vec4 = vec_env && atoi(vec_env) == 4;
    for (int attempt = try_vec4 ? 0 : 1; attempt < 2; ++attempt) {
        const Shape s = pick_shape(P.dim, attempt == 0);
        if (attempt == 0 && s.VEC != 4) continue;
        // split a positive's negatives over 4 lane groups when there are enough of them
        // (PT_STEP_S = 1 | 2 | 4 and PT_STEP_NCH override, for tuning)
        int S = (P.neg >= 8 && 256 / s.G >= 4) ? 4 : 1;
        if (const char *v = getenv("PT_STEP_S")) {
            const int want = atoi(v);
            if ((want == 1 || want == 2 || want == 4) && 256 / s.G >= want) S = want;
        }
        const int64_t nper = (P.neg + S - 1) / S;
        int nch = pick_nch(nper, s.KCH * s.VEC);
        if (const char *v = getenv("PT_STEP_NCH")) nch = atoi(v);
        // double-buffer the negative rows when a lane group takes more than one chunk (PT_STEP_DB=0 off)
        bool db = nper > nch;
        if (const char *v = getenv("PT_STEP_DB")) db = db && atoi(v) != 0;
        const int64_t gpb = 256 / s.G, ppb = gpb / S;
        const dim3 grid((unsigned)((P.batch_size + ppb - 1) / ppb)), block(256);
        size_t lds = (size_t)ppb * (size_t)P.neg * sizeof(int64_t) * (csr ? 2 : 1);
        if (S > 1) lds += sizeof(float) * ((size_t)gpb * 4 * s.KCH * s.G * s.VEC + (size_t)gpb * 2);
        if (lds > 64 * 1024) continue;
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
        for (int pass = 0; pass < 2; ++pass) {   // no double-buffered instance: single buffer
            PT_SSHAPES(PT_SSTEP)
            if (!db) break;
            db = false;
        }
#undef PT_SSTEP
    }
    return hipErrorInvalidValue;
}

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
    int64_t rows = 0;
    for (int i = 0; i < A.ntab; ++i) rows += A.t[i].rows;
    const int64_t gpb = 256 / s.G;
    // PT_APPLY_RPW=2|4: several rows per lane group with one contribution stream (measured slower on
    // C2: 20.4 / 22.0 us vs 16.8 us for one row per group, which stays the default)
    const char *rpw_env = getenv("PT_APPLY_RPW");
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

hipError_t launch_score(const StepParams &P, int mode, const int64_t *h, const int64_t *t, const int64_t *r, int64_t n,
                        float *out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const Shape s = pick_shape(P.dim);
    const int64_t gpb = 256 / s.G;
    const dim3 grid((unsigned)((n + gpb - 1) / gpb)), block(256);
#define PT_SCORE(G_, V_, K_)                                                                                     \
    if (s.G == G_ && s.VEC == V_ && s.KCH == K_) {                                                             \
        if (P.model == 0)                                                                                        \
            hipLaunchKernelGGL((dev::k_score<0, G_, V_, K_>), grid, block, 0, st, P, mode, h, t, r, n, out);     \
        else                                                                                                     \
            hipLaunchKernelGGL((dev::k_score<1, G_, V_, K_>), grid, block, 0, st, P, mode, h, t, r, n, out);     \
        return hipGetLastError();                                                                              \
    }
    PT_SHAPES(PT_SCORE)
#undef PT_SCORE
    return hipErrorInvalidValue;
}

hipError_t launch_score_queries(const StepParams &P, int side, const int64_t *qh, const int64_t *qt, const int64_t *qr,
                                int64_t nq, int64_t E, float *out, hipStream_t st, int global_order) {
    if (nq <= 0) return hipSuccess;
    const Shape s = pick_shape(P.dim);
    const int64_t gpb = 256 / s.G;
    int64_t bx = (E + gpb - 1) / gpb;
    if (bx > 128) bx = 128;
    const dim3 grid((unsigned)bx, (unsigned)nq), block(256);
#define PT_SQ(G_, V_, K_)                                                                                            \
    if (s.G == G_ && s.VEC == V_ && s.KCH == K_) {                                                                 \
        if (P.model == 0)                                                                                            \
            hipLaunchKernelGGL((dev::k_score_queries<0, G_, V_, K_>), grid, block, 0, st, P, side, qh, qt, qr, nq, E, \
                               out, global_order);                                                                   \
        else                                                                                                         \
            hipLaunchKernelGGL((dev::k_score_queries<1, G_, V_, K_>), grid, block, 0, st, P, side, qh, qt, qr, nq, E, \
                               out, global_order);                                                                   \
        return hipGetLastError();                                                                                  \
    }
    PT_SHAPES(PT_SQ)
#undef PT_SQ
    return hipErrorInvalidValue;
}

hipError_t launch_lp_min(const LpUniverseDev *us, const LpPair *pairs, int64_t n_pairs, const int64_t *uoff,
                         const int32_t *uids, int64_t n_active, int64_t dim, int64_t max_ent, int model, int p_norm,
                         int norm_flag, int64_t global_E, float *base, float *normal, float *rows, float *tuple_min,
                         hipStream_t st) {
    if (n_pairs <= 0) return hipSuccess;
    const Shape s = pick_shape(dim);
    const int64_t gpb = 256 / s.G;
    const dim3 gb((unsigned)((n_pairs + gpb - 1) / gpb)), block(256);
    int64_t bx = (max_ent + gpb * 4 - 1) / (gpb * 4);
    if (bx > 32) bx = 32;
    if (bx < 1) bx = 1;
#define PT_LP(G_, V_, K_)                                                                                          \
    if (s.G == G_ && s.VEC == V_ && s.KCH == K_) {                                                               \
        for (int64_t y0 = 0; y0 < n_active; y0 += 65535) {                                                         \
            const dim3 gs((unsigned)bx, (unsigned)(n_active - y0 < 65535 ? n_active - y0 : 65535));              \
            if (y0 == 0) {                                                                                         \
                if (model == 0)                                                                                    \
                    hipLaunchKernelGGL((dev::k_lp_bases<0, G_, V_, K_>), gb, block, 0, st, us, pairs, n_pairs,    \
                                       p_norm, norm_flag, base, normal, tuple_min);                                \
                else                                                                                               \
                    hipLaunchKernelGGL((dev::k_lp_bases<1, G_, V_, K_>), gb, block, 0, st, us, pairs, n_pairs,    \
                                       p_norm, norm_flag, base, normal, tuple_min);                                \
            }                                                                                                      \
            if (model == 0)                                                                                        \
                hipLaunchKernelGGL((dev::k_lp_scan<0, G_, V_, K_>), gs, block, 0, st, us, pairs, uoff, uids + y0,   \
                                   p_norm, norm_flag, global_E, base, normal, rows);                                \
            else                                                                                                   \
                hipLaunchKernelGGL((dev::k_lp_scan<1, G_, V_, K_>), gs, block, 0, st, us, pairs, uoff, uids + y0,   \
                                   p_norm, norm_flag, global_E, base, normal, rows);                                \
        }                                                                                                          \
        return hipGetLastError();                                                                                  \
    }
    PT_SHAPES(PT_LP)
#undef PT_LP
    return hipErrorInvalidValue;
}

}  // namespace pt
