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

#include "graph.h"
#include "kernels.h"
#include "rng.h"

namespace pt {
namespace dev {

constexpr float kEps = 1e-12f;   // F.normalize eps

// ---------------------------------------------------------------- lane-group vectors -----------
template <int G>
__device__ __forceinline__ float gsum(float v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, G);
    return v;
}

template <int G, int VEC, int KCH>
struct V {
    static constexpr int N = VEC * KCH;
    float x[N];
};

template <int G, int VEC, int KCH>
__device__ __forceinline__ void vload(V<G, VEC, KCH> &o, const float *__restrict__ row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if (c * VEC < D) {
            if constexpr (VEC == 4) {
                const float4 f = *reinterpret_cast<const float4 *>(row + c * 4);
                o.x[k * 4 + 0] = f.x; o.x[k * 4 + 1] = f.y; o.x[k * 4 + 2] = f.z; o.x[k * 4 + 3] = f.w;
            } else {
#pragma unroll
                for (int q = 0; q < VEC; ++q) o.x[k * VEC + q] = row[c * VEC + q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < VEC; ++q) o.x[k * VEC + q] = 0.f;
        }
    }
}

template <int G, int VEC, int KCH>
__device__ __forceinline__ void vstore(const V<G, VEC, KCH> &o, float *__restrict__ row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if (c * VEC < D) {
            if constexpr (VEC == 4) {
                *reinterpret_cast<float4 *>(row + c * 4) =
                    make_float4(o.x[k * 4 + 0], o.x[k * 4 + 1], o.x[k * 4 + 2], o.x[k * 4 + 3]);
            } else {
#pragma unroll
                for (int q = 0; q < VEC; ++q) row[c * VEC + q] = o.x[k * VEC + q];
            }
        }
    }
}

template <int G, int VEC, int KCH>
__device__ __forceinline__ void vatomic(const V<G, VEC, KCH> &o, float *__restrict__ row, int D, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        if (c * VEC < D) {
#pragma unroll
            for (int q = 0; q < VEC; ++q) atomicAdd(row + c * VEC + q, o.x[k * VEC + q]);
        }
    }
}

template <int G, int VEC, int KCH>
__device__ __forceinline__ float vdot(const V<G, VEC, KCH> &a, const V<G, VEC, KCH> &b) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) s += a.x[i] * b.x[i];
    return gsum<G>(s);
}

template <int G, int VEC, int KCH>
__device__ __forceinline__ void vzero(V<G, VEC, KCH> &a) {
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) a.x[i] = 0.f;
}

template <int G, int VEC, int KCH>
__device__ __forceinline__ bool vnonzero(const V<G, VEC, KCH> &a) {
    int nz = 0;
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) nz |= a.x[i] != 0.f;
    return gsum<G>((float)nz) != 0.f;
}

// F.normalize(x, 2, -1): out = x / max(||x||, eps); returns ||x||
template <int G, int VEC, int KCH>
__device__ __forceinline__ float vnormalize(const V<G, VEC, KCH> &x, V<G, VEC, KCH> &out) {
    const float n = sqrtf(vdot(x, x));
    const float den = n > kEps ? n : kEps;
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) out.x[i] = x.x[i] / den;
    return n;
}

// backward of F.normalize at raw x with norm n: (g - x (x.g)/n^2) / n   (clamp_min branch: g / eps)
template <int G, int VEC, int KCH>
__device__ __forceinline__ void vnormalize_bwd(const V<G, VEC, KCH> &x, float n, const V<G, VEC, KCH> &g,
                                               V<G, VEC, KCH> &out) {
    if (n > kEps) {
        const float c = vdot(g, x) / (n * n);
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) out.x[i] = (g.x[i] - x.x[i] * c) / n;
    } else {
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) out.x[i] = g.x[i] / kEps;
    }
}

// ||v||_p for p in {1,2}
template <int G, int VEC, int KCH>
__device__ __forceinline__ float vpnorm(const V<G, VEC, KCH> &v, int p) {
    float s = 0.f;
    if (p == 1) {
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) s += fabsf(v.x[i]);
        return gsum<G>(s);
    }
#pragma unroll
    for (int i = 0; i < V<G, VEC, KCH>::N; ++i) s += v.x[i] * v.x[i];
    return sqrtf(gsum<G>(s));
}

// ds * d||v||_p/dv : p=1 sgn(v)*ds (sgn 0 = 0), p=2 v*(ds/||v||) masked at ||v|| = 0
template <int G, int VEC, int KCH>
__device__ __forceinline__ void vpnorm_bwd(const V<G, VEC, KCH> &v, float nv, int p, float ds, V<G, VEC, KCH> &g) {
    if (p == 1) {
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) g.x[i] = v.x[i] > 0.f ? ds : (v.x[i] < 0.f ? -ds : 0.f);
    } else {
        const float k = nv == 0.f ? 0.f : ds / nv;
#pragma unroll
        for (int i = 0; i < V<G, VEC, KCH>::N; ++i) g.x[i] = v.x[i] * k;
    }
}

// ---------------------------------------------------------------- sampler --------------------
__device__ __forceinline__ int64_t rand_max(uint64_t &s, int64_t x) { return (int64_t)(lcg_next(s) % (uint64_t)x); }

// Filtered corruption (Corrupt.h:27-56 / :75-104): `vals` is the searched column of the sorted list
// (trainHead[].t for corrupt_head, trainTail[].h for corrupt_tail) and [lo, hi] the run of known
// partners of the positive's (entity, relation) - the [ll, rr] of the reference's two binary searches,
// precomputed per triple (TripleRec). The draw and the final search are the reference's.
__device__ __forceinline__ int64_t corrupt_in_run(const int32_t *__restrict__ vals, int64_t lo, int64_t hi, int64_t E,
                                                  uint64_t &s) {
    const int64_t tmp = rand_max(s, E - (hi - lo + 1));
    if (tmp < vals[lo]) return tmp;
    if (tmp > vals[hi] - hi + lo - 1) return tmp + hi - lo + 1;
    int64_t l = lo, r = hi + 1;
    while (l + 1 < r) {
        const int64_t mid = (l + r) >> 1;
        if (vals[mid] - mid + lo - 1 < tmp) l = mid; else r = mid;
    }
    return tmp + l - lo + 1;
}

// state of the sampler stream that produces positive b of this call (Base.cpp:200-207 split)
__device__ __forceinline__ uint64_t positive_state(const uint64_t *states, int64_t threads, int64_t bs, int64_t b,
                                                   int64_t dpp) {
    const int64_t per = bs % threads == 0 ? bs / threads : bs / threads + 1;
    const int64_t id = b / per;
    return lcg_jump(states[id], (uint64_t)((b - id * per) * dpp));
}

struct PosDraw {
    int64_t h, r, t;
    int32_t hr_lo, hr_hi, tr_lo, tr_hi;
    uint64_t s1;   // stream state after the positive's index draw
};

// positive b: i = rand_max(trainTotal), trainList[i] (Base.cpp:210-215)
__device__ __forceinline__ PosDraw draw_positive(const DeviceGraph &g, const uint64_t *states, int64_t threads,
                                                 int64_t bs, int64_t b, int64_t dpp) {
    uint64_t s = positive_state(states, threads, bs, b, dpp);
    const int64_t i = rand_max(s, g.train_total);
    const int4 *p = reinterpret_cast<const int4 *>(g.rec + i);
    const int4 a = p[0], c = p[1];
    return PosDraw{a.x, a.y, a.z, a.w, c.x, c.y, c.z, s};
}

// negative k of a positive (stream offsets 1+2k coin, 2+2k corruption; Base.cpp:217-232): returns the
// corrupted entity, *tail_side = 1 when the tail was replaced (corrupt_head), 0 when the head was
__device__ __forceinline__ int64_t draw_negative(const DeviceGraph &g, const PosDraw &p, int64_t k, int bern,
                                                 int filter, int *tail_side) {
    uint64_t s = lcg_jump(p.s1, (uint64_t)(2 * k));
    const float prob = bern ? g.bern_prob[p.r] : 500.f;
    const int64_t E = g.ent_total;
    if ((float)(lcg_next(s) % 1000ULL) < prob) {
        *tail_side = 1;
        if (filter) return corrupt_in_run(g.head_t, p.hr_lo, p.hr_hi, E, s);
        const int64_t tmp = rand_max(s, E - 1);   // skips the passed entity h (Corrupt.h:18-25)
        return tmp < p.h ? tmp : tmp + 1;
    }
    *tail_side = 0;
    if (filter) return corrupt_in_run(g.tail_h, p.tr_lo, p.tr_hi, E, s);
    const int64_t tmp = rand_max(s, E - 1);       // skips t (Corrupt.h:68-74)
    return tmp < p.t ? tmp : tmp + 1;
}

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

__device__ __forceinline__ void advance_states(uint64_t *states, int64_t threads, int64_t bs, int64_t dpp, int lane) {
    if (lane < threads) {
        const int64_t per = bs % threads == 0 ? bs / threads : bs / threads + 1;
        int64_t len = bs - lane * per;
        len = len < 0 ? 0 : (len > per ? per : len);
        states[lane] = lcg_jump(states[lane], (uint64_t)(len * dpp));
    }
}

__global__ void k_advance(uint64_t *states, int64_t threads, int64_t bs, int64_t dpp) {
    advance_states(states, threads, bs, dpp, (int)threadIdx.x);
}

// ---------------------------------------------------------------- fused step -----------------
// Gradient sink of the single-model path: memory-side float atomics into per-table gradient rows,
// plus a touched-row flag for the sparse apply pass.
struct GlobalSink {
    float *gent, *grel, *gnorm;
    int *fent, *frel, *fnorm;
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

// One positive group: forward + MarginLoss + backward for the positive and its `neg` negatives.
// Gradient conventions per table (the apply pass finishes them):
//   TransE: ent and rel gradients in normalized space (the apply pass multiplies by the normalize
//           Jacobian of the pre-step row; sum-then-Jacobian == Jacobian-then-sum, it is linear);
//   TransH: ent gradients raw (their projection/normalize Jacobians depend on the relation, so they are
//           applied here), rel in normalized space, norm_vector in normalized (n-hat) space.
// Negatives are given by `get_neg(k, &h, &t, &r)`; rows equal to the positive's reuse its registers
// and accumulate on chip, other rows go straight to the sink.
template <int MODEL, int G, int VEC, int KCH, typename Sink, typename NegFn>
__device__ __forceinline__ float group_step(const StepParams &P, int64_t hp, int64_t rp, int64_t tp, int64_t neg,
                                            NegFn get_neg, const Sink &sink, int lane) {
    using Vec = V<G, VEC, KCH>;
    const int D = (int)P.dim;
    const int p = P.p_norm;
    const bool nf = P.norm_flag != 0;
    // ---- positive
    Vec H, T, Rr, W, nW, hh, th, rh, vpos;
    float hn = 0, tn = 0, hdot = 0, tdot = 0;
    vload(H, P.ent + hp * D, D, lane);
    vload(T, P.ent + tp * D, D, lane);
    vload(Rr, P.rel + rp * D, D, lane);
    Vec Hs = H, Ts = T;   // scored entity vectors (projected for TransH)
    if constexpr (MODEL == 1) {
        vload(W, P.normv + rp * D, D, lane);
        vnormalize(W, nW);
        hdot = vdot(H, nW);
        tdot = vdot(T, nW);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            Hs.x[i] = H.x[i] - hdot * nW.x[i];
            Ts.x[i] = T.x[i] - tdot * nW.x[i];
        }
    }
    if (nf) {
        hn = vnormalize(Hs, hh);
        vnormalize(Rr, rh);
        tn = vnormalize(Ts, th);
    } else {
        hh = Hs; rh = Rr; th = Ts;
    }
#pragma unroll
    for (int i = 0; i < Vec::N; ++i) vpos.x[i] = (hh.x[i] + rh.x[i]) - th.x[i];
    const float ps = vpnorm(vpos, p);

    Vec aH, aT, aR, aW;   // on-chip accumulators of the positive's rows
    vzero(aH); vzero(aT); vzero(aR); vzero(aW);
    float csum = 0.f, lsum = 0.f;
    const float m = P.margin;
    const float inv = P.inv_count;

    for (int64_t k = 0; k < neg; ++k) {
        int64_t hk, tk, rk;
        get_neg(k, hk, tk, rk);
        const bool same_r = rk == rp;
        // relation row of the negative
        Vec Rk, rkh, Wk, nWk;
        if (same_r) {
            rkh = rh;
            if constexpr (MODEL == 1) { nWk = nW; Wk = W; }
        } else {
            vload(Rk, P.rel + rk * D, D, lane);
            if (nf) vnormalize(Rk, rkh); else rkh = Rk;
            if constexpr (MODEL == 1) {
                vload(Wk, P.normv + rk * D, D, lane);
                vnormalize(Wk, nWk);
            }
        }
        // entity rows of the negative: reuse the positive's when the (row, relation) matches
        Vec Ek[2], Eks[2], ekh[2];
        float ekn[2], ekdot[2];
        int role[2];   // 0: row hp, 1: row tp, -1: other
        const int64_t ids[2] = {hk, tk};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int64_t e = ids[s];
            role[s] = !same_r ? -1 : (e == hp ? 0 : (e == tp ? 1 : -1));
            if (role[s] == 0) {
                Ek[s] = H; Eks[s] = Hs; ekh[s] = hh; ekn[s] = hn; ekdot[s] = hdot;
            } else if (role[s] == 1) {
                Ek[s] = T; Eks[s] = Ts; ekh[s] = th; ekn[s] = tn; ekdot[s] = tdot;
            } else {
                vload(Ek[s], P.ent + e * D, D, lane);
                Eks[s] = Ek[s];
                ekdot[s] = 0.f;
                if constexpr (MODEL == 1) {
                    ekdot[s] = vdot(Ek[s], nWk);
#pragma unroll
                    for (int i = 0; i < Vec::N; ++i) Eks[s].x[i] = Ek[s].x[i] - ekdot[s] * nWk.x[i];
                }
                if (nf) ekn[s] = vnormalize(Eks[s], ekh[s]); else { ekh[s] = Eks[s]; ekn[s] = 0.f; }
            }
        }
        Vec vk;
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) vk.x[i] = (ekh[0].x[i] + rkh.x[i]) - ekh[1].x[i];
        const float ns = vpnorm(vk, p);
        const float a = ps - ns;
        lsum += a > -m ? a : -m;
        const float c = a > -m ? inv : (a == -m ? inv * 0.5f : 0.f);
        if (c == 0.f) continue;
        csum += c;
        Vec g;
        vpnorm_bwd(vk, ns, p, -c, g);   // d loss / d v_k
        // relation (normalized space)
        if (same_r) {
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) aR.x[i] += g.x[i];
        } else {
            sink.rel(rk, g, D, lane);
        }
        Vec gw;   // TransH: d/d n-hat of this negative's relation
        if constexpr (MODEL == 1) vzero(gw);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            Vec gs;   // d/d(normalized scored entity): +g for the head, -g for the tail
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) gs.x[i] = s == 0 ? g.x[i] : -g.x[i];
            if (role[s] >= 0) {
                Vec &acc = role[s] == 0 ? aH : aT;
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) acc.x[i] += gs.x[i];
                continue;
            }
            if constexpr (MODEL == 0) {
                sink.ent(ids[s], gs, D, lane);
            } else {
                Vec gp;   // through normalize of the projected vector
                if (nf) vnormalize_bwd(Eks[s], ekn[s], gs, gp); else gp = gs;
                const float ng = vdot(nWk, gp);
                Vec ge;
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) {
                    ge.x[i] = gp.x[i] - nWk.x[i] * ng;
                    gw.x[i] -= ekdot[s] * gp.x[i] + ng * Ek[s].x[i];
                }
                sink.ent(ids[s], ge, D, lane);
            }
        }
        if constexpr (MODEL == 1) {
            if (same_r) {
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) aW.x[i] += gw.x[i];
            } else if (vnonzero(gw)) {
                sink.norm(rk, gw, D, lane);
            }
        }
    }
    // ---- positive backward
    if (csum != 0.f) {
        Vec g;
        vpnorm_bwd(vpos, ps, p, csum, g);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            aH.x[i] += g.x[i];
            aR.x[i] += g.x[i];
            aT.x[i] -= g.x[i];
        }
    }
    if (vnonzero(aR)) sink.rel(rp, aR, D, lane);
    if constexpr (MODEL == 0) {
        if (vnonzero(aH)) sink.ent(hp, aH, D, lane);
        if (vnonzero(aT)) sink.ent(tp, aT, D, lane);
    } else {
        // positive-row accumulators are in normalized-projected space: finish them once
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            Vec &acc = s == 0 ? aH : aT;
            if (!vnonzero(acc)) continue;
            const Vec &E = s == 0 ? H : T;
            const Vec &Es = s == 0 ? Hs : Ts;
            const float en = s == 0 ? hn : tn;
            const float edot = s == 0 ? hdot : tdot;
            Vec gp;
            if (nf) vnormalize_bwd(Es, en, acc, gp); else gp = acc;
            const float ng = vdot(nW, gp);
            Vec ge;
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) {
                ge.x[i] = gp.x[i] - nW.x[i] * ng;
                aW.x[i] -= edot * gp.x[i] + ng * E.x[i];
            }
            sink.ent(s == 0 ? hp : tp, ge, D, lane);
        }
        if (vnonzero(aW)) sink.norm(rp, aW, D, lane);
    }
    return lsum;
}

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
    if (lane == 0 && loss) atomicAdd(loss, lsum * P.inv_count);
}

// Fused step with in-kernel sampling (the Trainer.run hot loop). One lane group per positive; the
// group's negatives are drawn lane-parallel into LDS, then EVERY row the group needs is loaded
// before the first gradient atomic is issued (s_waitcnt vmcnt counts loads and atomics in issue
// order, so a load behind an atomic would wait for it), NCH negative rows held in registers.
// Rows use the VEC=1 layout so each atomic wave-instruction covers 64 contiguous floats.
template <int MODEL, int G, int KCH, int NCH>
__global__ __launch_bounds__(256) void k_step_sampled(StepParams P, DeviceGraph g, const uint64_t *__restrict__ states,
                                                      int64_t threads, int bern, int filter, GlobalSink sink,
                                                      float *__restrict__ loss) {
    using Vec = V<G, 1, KCH>;
    constexpr int GPB = 256 / G;
    extern __shared__ __attribute__((aligned(16))) int64_t s_neg[];   // [GPB][neg] (entity << 1 | tail_side)
    const int lane = threadIdx.x % G;
    const int grp = threadIdx.x / G;
    const int64_t bs = P.batch_size, neg = P.neg;
    const int64_t b = (int64_t)blockIdx.x * GPB + grp;
    const bool active = b < bs;
    PosDraw pd{};
    if (active) {
        pd = draw_positive(g, states, threads, bs, b, 1 + 2 * neg);
        for (int64_t k = lane; k < neg; k += G) {
            int side;
            const int64_t e = draw_negative(g, pd, k, bern, filter, &side);
            s_neg[grp * neg + k] = (e << 1) | side;
        }
    }
    __syncthreads();
    if (!active) return;
    const int64_t *mine = s_neg + grp * neg;
    const int D = (int)P.dim;
    const int p = P.p_norm;
    const bool nf = P.norm_flag != 0;
    const int64_t hp = pd.h, rp = pd.r, tp = pd.t;
    Vec H, T, Rr, W, nW, hh, th, rh, vpos;
    vload(H, P.ent + hp * D, D, lane);
    vload(T, P.ent + tp * D, D, lane);
    vload(Rr, P.rel + rp * D, D, lane);
    if constexpr (MODEL == 1) vload(W, P.normv + rp * D, D, lane);
    Vec E[NCH];
    auto load_chunk = [&](int64_t c0) {
#pragma unroll
        for (int k = 0; k < NCH; ++k)
            if (c0 + k < neg) vload(E[k], P.ent + (mine[c0 + k] >> 1) * D, D, lane);
    };
    load_chunk(0);
    // ---- positive forward
    Vec Hs = H, Ts = T;
    float hn = 0, tn = 0, hdot = 0, tdot = 0;
    if constexpr (MODEL == 1) {
        vnormalize(W, nW);
        hdot = vdot(H, nW);
        tdot = vdot(T, nW);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            Hs.x[i] = H.x[i] - hdot * nW.x[i];
            Ts.x[i] = T.x[i] - tdot * nW.x[i];
        }
    }
    if (nf) {
        hn = vnormalize(Hs, hh);
        vnormalize(Rr, rh);
        tn = vnormalize(Ts, th);
    } else {
        hh = Hs; rh = Rr; th = Ts;
    }
#pragma unroll
    for (int i = 0; i < Vec::N; ++i) vpos.x[i] = (hh.x[i] + rh.x[i]) - th.x[i];
    const float ps = vpnorm(vpos, p);
    Vec aH, aT, aR, aW;
    vzero(aH); vzero(aT); vzero(aR); vzero(aW);
    float csum = 0.f, lsum = 0.f;
    const float m = P.margin, inv = P.inv_count;
    for (int64_t c0 = 0;;) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            if (c0 + k >= neg) break;
            const int64_t v = mine[c0 + k];
            const int64_t e = v >> 1;
            const bool tail_side = v & 1;
            Vec Es = E[k], eh, vk;
            float ed = 0.f, en = 0.f;
            if constexpr (MODEL == 1) {
                ed = vdot(E[k], nW);
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) Es.x[i] = E[k].x[i] - ed * nW.x[i];
            }
            if (nf) en = vnormalize(Es, eh); else eh = Es;
#pragma unroll
            for (int i = 0; i < Vec::N; ++i)
                vk.x[i] = tail_side ? (hh.x[i] + rh.x[i]) - eh.x[i] : (eh.x[i] + rh.x[i]) - th.x[i];
            const float ns = vpnorm(vk, p);
            const float a = ps - ns;
            lsum += a > -m ? a : -m;
            const float c = a > -m ? inv : (a == -m ? inv * 0.5f : 0.f);
            if (c == 0.f) continue;
            csum += c;
            Vec gk, gs;
            vpnorm_bwd(vk, ns, p, -c, gk);
#pragma unroll
            for (int i = 0; i < Vec::N; ++i) {
                aR.x[i] += gk.x[i];
                if (tail_side) aH.x[i] += gk.x[i]; else aT.x[i] -= gk.x[i];
                gs.x[i] = tail_side ? -gk.x[i] : gk.x[i];   // corrupted tail gets -g, corrupted head +g
            }
            if constexpr (MODEL == 0) {
                sink.ent(e, gs, D, lane);
            } else {
                Vec gp, ge;
                if (nf) vnormalize_bwd(Es, en, gs, gp); else gp = gs;
                const float ng = vdot(nW, gp);
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) {
                    ge.x[i] = gp.x[i] - nW.x[i] * ng;
                    aW.x[i] -= ed * gp.x[i] + ng * E[k].x[i];
                }
                sink.ent(e, ge, D, lane);
            }
        }
        c0 += NCH;
        if (c0 >= neg) break;
        load_chunk(c0);
    }
    // ---- positive backward and the group's on-chip accumulators
    if (csum != 0.f) {
        Vec gv;
        vpnorm_bwd(vpos, ps, p, csum, gv);
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            aH.x[i] += gv.x[i];
            aR.x[i] += gv.x[i];
            aT.x[i] -= gv.x[i];
        }
        sink.rel(rp, aR, D, lane);
        if constexpr (MODEL == 0) {
            sink.ent(hp, aH, D, lane);
            sink.ent(tp, aT, D, lane);
        } else {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const Vec &acc = s2 == 0 ? aH : aT;
                const Vec &Ev = s2 == 0 ? H : T;
                const Vec &Esv = s2 == 0 ? Hs : Ts;
                const float enn = s2 == 0 ? hn : tn;
                const float edd = s2 == 0 ? hdot : tdot;
                Vec gp, ge;
                if (nf) vnormalize_bwd(Esv, enn, acc, gp); else gp = acc;
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
    if (lane == 0 && loss) atomicAdd(loss, lsum * inv);
}

// Sparse apply: for every touched row finish the gradient (normalize Jacobian of the pre-step row
// when that table's gradient is in normalized space) and run SGD / Adagrad; then clear the row.
struct ApplyTable {
    float *w, *acc, *grad;
    int *flag;
    int64_t rows;
    int jacobian;
};
struct ApplyParams {
    ApplyTable t[3];
    int ntab;
    int64_t dim;
    int opt;
    float lr;
    // sampler advance + loss margin (done by block 0)
    uint64_t *states;
    int64_t threads, bs, dpp;
    float *loss;
    float margin;
};

template <int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_apply(ApplyParams A) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    const int lane = threadIdx.x % G;
    int64_t row = (int64_t)blockIdx.x * GPB + threadIdx.x / G;
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        if (A.states) advance_states(A.states, A.threads, A.bs, A.dpp, (int)threadIdx.x);
        if (A.loss && threadIdx.x == 0) *A.loss += A.margin;
    }
    int ti = 0;
    while (ti < A.ntab && row >= A.t[ti].rows) {
        row -= A.t[ti].rows;
        ++ti;
    }
    if (ti >= A.ntab) return;
    const ApplyTable &T = A.t[ti];
    if (!T.flag[row]) return;
    const int D = (int)A.dim;
    Vec x, gsum_, g;
    vload(x, T.w + row * D, D, lane);
    vload(gsum_, T.grad + row * D, D, lane);
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
    Vec z;
    vzero(z);
    vstore(z, T.grad + row * D, D, lane);
    if (lane == 0) T.flag[row] = 0;
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
                                                       int64_t nq, int64_t E, float *__restrict__ out) {
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
        const int64_t e = j == 0 ? truth : (j - 1 < truth ? j - 1 : j);
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
// For a (key, universe) pair: score every local entity of the universe as the missing side and MIN
// it into the key's global score row (scores are norms >= 0, so float order == int order).
template <int MODEL, int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_lp_min(const LpUniverseDev *__restrict__ us, const LpPair *__restrict__ pairs,
                                                int64_t n_pairs, int p_norm, int norm_flag, int64_t global_E,
                                                float *__restrict__ rows) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = 256 / G;
    const int lane = threadIdx.x % G;
    const int grp = threadIdx.x / G;
    const int64_t pi = blockIdx.y;
    if (pi >= n_pairs) return;
    const LpPair pr = pairs[pi];
    const LpUniverseDev U = us[pr.universe];
    const int D = (int)U.dim;
    Vec A, R, ah, rh, nW;
    vload(A, U.ent + (int64_t)pr.anchor * D, D, lane);
    vload(R, U.rel + (int64_t)pr.rel * D, D, lane);
    float adot = 0.f;
    if constexpr (MODEL == 1) {
        Vec W;
        vload(W, U.normv + (int64_t)pr.rel * D, D, lane);
        vnormalize(W, nW);
        adot = vdot(A, nW);
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) A.x[k] = A.x[k] - adot * nW.x[k];
    }
    if (norm_flag) {
        vnormalize(A, ah);
        vnormalize(R, rh);
    } else {
        ah = A; rh = R;
    }
    // head prediction: score = e + (r - t); tail prediction: (h + r) - e   (TransE.py:56-59)
    Vec base;
#pragma unroll
    for (int k = 0; k < Vec::N; ++k) base.x[k] = pr.side == 1 ? rh.x[k] - ah.x[k] : ah.x[k] + rh.x[k];
    float *out = rows + (int64_t)pr.key * global_E;
    for (int64_t e = (int64_t)blockIdx.x * GPB + grp; e < U.ent_total; e += (int64_t)gridDim.x * GPB) {
        Vec X, xh, v;
        vload(X, U.ent + e * D, D, lane);
        if constexpr (MODEL == 1) {
            const float xd = vdot(X, nW);
#pragma unroll
            for (int k = 0; k < Vec::N; ++k) X.x[k] = X.x[k] - xd * nW.x[k];
        }
        if (norm_flag) vnormalize(X, xh); else xh = X;
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) v.x[k] = pr.side == 1 ? xh.x[k] + base.x[k] : base.x[k] - xh.x[k];
        const float s = vpnorm(v, p_norm);
        if (lane == 0) atomicMin(reinterpret_cast<int *>(out + U.remap[e]), __float_as_int(s));
    }
}

}  // namespace dev

// ==================================================================== host launchers ===========
namespace {

struct Shape {
    int G, VEC, KCH;
};

Shape pick_shape(int64_t D, bool vec4 = true) {
    const int VEC = vec4 && D % 4 == 0 ? 4 : 1;
    const int64_t chunks = D / VEC;
    int G = 1;
    while (G < chunks && G < 64) G <<= 1;
    if (G < 2) G = 2;
    int KCH = (int)((chunks + G - 1) / G);
    if (VEC == 1) {   // VEC=1 instantiations exist for power-of-two chunk counts
        int k = 1;
        while (k < KCH) k <<= 1;
        KCH = k;
    }
    return Shape{G, VEC, KCH};
}

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

#define PT_SHAPES(X)                                                                                  \
    X(2, 4, 1) X(4, 4, 1) X(8, 4, 1) X(16, 4, 1) X(32, 4, 1) X(64, 4, 1) X(64, 4, 2)                 \
    X(2, 1, 1) X(4, 1, 1) X(8, 1, 1) X(16, 1, 1) X(32, 1, 1) X(64, 1, 1) X(64, 1, 2) X(64, 1, 4)    \
    X(64, 1, 8)

// VEC=1 shapes x NCH of the sampled step kernel
#define PT_SSHAPES(X)                                                                                 \
    X(2, 1, 1) X(2, 1, 4) X(2, 1, 8) X(2, 1, 32) X(4, 1, 1) X(4, 1, 4) X(4, 1, 8) X(4, 1, 32)         \
    X(8, 1, 1) X(8, 1, 4) X(8, 1, 8) X(8, 1, 32) X(16, 1, 1) X(16, 1, 4) X(16, 1, 8) X(16, 1, 32)     \
    X(32, 1, 1) X(32, 1, 4) X(32, 1, 8) X(32, 1, 32) X(64, 1, 1) X(64, 1, 4) X(64, 1, 8) X(64, 1, 32) \
    X(64, 2, 1) X(64, 2, 4) X(64, 2, 8) X(64, 2, 32) X(64, 4, 1) X(64, 4, 4) X(64, 4, 8) X(64, 4, 32) \
    X(64, 8, 1) X(64, 8, 4) X(64, 8, 8)

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

hipError_t launch_sample(const DeviceGraph &g, const uint64_t *states, int64_t threads, int64_t bs, int64_t neg,
                         int bern, int filter, int64_t *h, int64_t *t, int64_t *r, float *y, hipStream_t st) {
    if (bs <= 0) return hipSuccess;
    const int bl = 256;
    hipLaunchKernelGGL(dev::k_sample, dim3((unsigned)((bs + bl - 1) / bl)), dim3(bl), 0, st, g, states, threads, bs,
                       neg, bern, filter, h, t, r, y);
    return hipGetLastError();
}

hipError_t launch_advance(uint64_t *states, int64_t threads, int64_t bs, int64_t dpp, hipStream_t st) {
    hipLaunchKernelGGL(dev::k_advance, dim3(1), dim3(64), 0, st, states, threads, bs, dpp);
    return hipGetLastError();
}

hipError_t launch_step(const StepParams &P, const DeviceGraph &g, const uint64_t *states, int64_t threads, int bern,
                       int filter, const int64_t *bh, const int64_t *bt, const int64_t *br, const StepWorkspace &W,
                       float *loss, hipStream_t st) {
    if (P.batch_size <= 0) return hipSuccess;
    dev::GlobalSink sink{W.gent, W.grel, W.gnorm, W.fent, W.frel, W.fnorm};
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
    const Shape s = pick_shape(P.dim, false);
    const int nch = pick_nch(P.neg, s.KCH);
    const int64_t gpb = 256 / s.G;
    const dim3 grid((unsigned)((P.batch_size + gpb - 1) / gpb)), block(256);
    const size_t lds = (size_t)gpb * (size_t)P.neg * sizeof(int64_t);
#define PT_SSTEP(G_, K_, N_)                                                                                      \
    if (s.G == G_ && s.KCH == K_ && nch == N_) {                                                                \
        if (P.model == 0)                                                                                         \
            hipLaunchKernelGGL((dev::k_step_sampled<0, G_, K_, N_>), grid, block, lds, st, P, g, states, threads,  \
                               bern, filter, sink, loss);                                                         \
        else                                                                                                      \
            hipLaunchKernelGGL((dev::k_step_sampled<1, G_, K_, N_>), grid, block, lds, st, P, g, states, threads,  \
                               bern, filter, sink, loss);                                                         \
        return hipGetLastError();                                                                                 \
    }
    PT_SSHAPES(PT_SSTEP)
#undef PT_SSTEP
    return hipErrorInvalidValue;
}

hipError_t launch_apply(const StepParams &P, const StepWorkspace &W, uint64_t *states, int64_t threads, int64_t bs,
                        int64_t dpp, float *loss, hipStream_t st) {
    const Shape s = pick_shape(P.dim);
    dev::ApplyParams A{};
    A.ntab = 0;
    const int ent_j = P.model == 0 && P.norm_flag;
    A.t[A.ntab++] = dev::ApplyTable{P.ent, P.ent_acc, W.gent, W.fent, P.ent_total, ent_j};
    A.t[A.ntab++] = dev::ApplyTable{P.rel, P.rel_acc, W.grel, W.frel, P.rel_total, P.norm_flag};
    if (P.model == 1) A.t[A.ntab++] = dev::ApplyTable{P.normv, P.norm_acc, W.gnorm, W.fnorm, P.rel_total, 1};
    A.dim = P.dim;
    A.opt = P.opt;
    A.lr = P.lr;
    A.states = states;
    A.threads = threads;
    A.bs = bs;
    A.dpp = dpp;
    A.loss = loss;
    A.margin = P.margin;
    int64_t rows = 0;
    for (int i = 0; i < A.ntab; ++i) rows += A.t[i].rows;
    const int64_t gpb = 256 / s.G;
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
                                int64_t nq, int64_t E, float *out, hipStream_t st) {
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
                               out);                                                                                 \
        else                                                                                                         \
            hipLaunchKernelGGL((dev::k_score_queries<1, G_, V_, K_>), grid, block, 0, st, P, side, qh, qt, qr, nq, E, \
                               out);                                                                                 \
        return hipGetLastError();                                                                                  \
    }
    PT_SHAPES(PT_SQ)
#undef PT_SQ
    return hipErrorInvalidValue;
}

hipError_t launch_lp_min(const LpUniverseDev *us, const LpPair *pairs, int64_t n_pairs, int64_t dim, int64_t max_ent,
                         int model, int p_norm, int norm_flag, int64_t global_E, float *rows, hipStream_t st) {
    if (n_pairs <= 0) return hipSuccess;
    const Shape s = pick_shape(dim);
    const int64_t gpb = 256 / s.G;
    int64_t bx = (max_ent + gpb - 1) / gpb;
    if (bx > 64) bx = 64;
    if (bx < 1) bx = 1;
    const dim3 grid((unsigned)bx, (unsigned)n_pairs), block(256);
#define PT_LP(G_, V_, K_)                                                                                         \
    if (s.G == G_ && s.VEC == V_ && s.KCH == K_) {                                                              \
        if (model == 0)                                                                                           \
            hipLaunchKernelGGL((dev::k_lp_min<0, G_, V_, K_>), grid, block, 0, st, us, pairs, n_pairs, p_norm,    \
                               norm_flag, global_E, rows);                                                        \
        else                                                                                                      \
            hipLaunchKernelGGL((dev::k_lp_min<1, G_, V_, K_>), grid, block, 0, st, us, pairs, n_pairs, p_norm,    \
                               norm_flag, global_E, rows);                                                        \
        return hipGetLastError();                                                                               \
    }
    PT_SHAPES(PT_LP)
#undef PT_LP
    return hipErrorInvalidValue;
}

}  // namespace pt
