// Reference-order ("deterministic") training step: the gradient of every table row is summed in slot
// order, lookup by lookup, as torch's autograd does it for Trainer.train_one_step (Trainer.py:44-56):
// embedding_dense_backward per lookup (batch_h, batch_t, batch_r, and norm_vector(batch_r) for TransH)
// accumulates the slots' rows in slot order, AccumulateGrad adds the two entity lookups' dense
// gradients, then the dense SGD / Adagrad step (Trainer.py:62-88) changes every row with a gradient.
//
// The fast kernels (step.hip, apply.hip, universes.hip) sum the same contributions in arrival order
// (float atomics, LDS-linked contribution lists) and in normalized space; this path fixes the order and
// the arithmetic instead: sequential dot products and norms, IEEE division and square root, no fused
// multiply-add contraction (this translation unit compiles with contraction off). It is bit-identical
// run to run, and bit-identical to the CPU restatement in oracle/oracle.c (same order, same operations).
// It is the parity mode, selected per trainer / universe set (pt_trainer_set_deterministic,
// pt_universe_set_deterministic); its cost is a few passes per slot, not the fast path's single pass.
//
// Phases of one step (single model, grid-wide; universes: the same phases inside one workgroup):
//   score   every slot's score with the pre-step tables (TransE.py:46-74, TransH.py:52-93)
//   coef    MarginLoss coefficients per (positive, negative) (MarginLoss.py:24-28, NegativeSampling.py:13-31)
//   loss    the loss summed in (positive, negative) order in double (one lane)
//   grad    per slot with a nonzero coefficient its gradient rows per lookup
//   reduce  per table row: its slots' rows in slot order per lookup, the entity lookups added, update
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device.h"
#include "kernels.h"
#include "ordered.h"
#include "universes.h"

namespace pt {
namespace dev {

__device__ __forceinline__ float o_div(float a, float b) { return a / b; }   // IEEE (HIP default: correctly rounded)
__device__ __forceinline__ float o_sqrt(float a) { return __builtin_sqrtf(a); }   // IEEE, correctly rounded

// one slot's forward values (oracle.c slot_forward); element-wise intermediates are recomputed on demand
// with the same operations, so every value equals the oracle's materialized one
struct OSlot {
    const float *he, *te, *re, *we;
    int64_t d;
    int model, p, nf;
    float wn = 0.f, dw = 1.f, hdot = 0.f, tdot = 0.f;   // TransH: ||w||, max(||w||, eps), e . n-hat
    float hpn = 0.f, tpn = 0.f, rn = 0.f;              // norms of the (projected) h, t and of r
    float dh = 1.f, dt = 1.f, dr = 1.f;                // their max(norm, 1e-12)
    float sc = 0.f;

    __device__ __forceinline__ float nw(int64_t i) const { return o_div(we[i], dw); }
    __device__ __forceinline__ float hp(int64_t i) const { return model ? he[i] - hdot * nw(i) : he[i]; }
    __device__ __forceinline__ float tp(int64_t i) const { return model ? te[i] - tdot * nw(i) : te[i]; }
    __device__ __forceinline__ float nh(int64_t i) const { return nf ? o_div(hp(i), dh) : hp(i); }
    __device__ __forceinline__ float nt(int64_t i) const { return nf ? o_div(tp(i), dt) : tp(i); }
    __device__ __forceinline__ float nr(int64_t i) const { return nf ? o_div(re[i], dr) : re[i]; }
    __device__ __forceinline__ float v(int64_t i) const { return (nh(i) + nr(i)) - nt(i); }

    __device__ void forward() {
        if (model) {
            float s = 0.f;
            for (int64_t i = 0; i < d; ++i) s += we[i] * we[i];
            wn = o_sqrt(s);
            dw = wn > 1e-12f ? wn : 1e-12f;
            float a = 0.f, b = 0.f;
            for (int64_t i = 0; i < d; ++i) {
                const float n = nw(i);
                a += he[i] * n;
                b += te[i] * n;
            }
            hdot = a;
            tdot = b;
        }
        if (nf) {
            float a = 0.f, b = 0.f, c = 0.f;
            for (int64_t i = 0; i < d; ++i) {
                const float x = hp(i), y = tp(i);
                a += x * x;
                b += re[i] * re[i];
                c += y * y;
            }
            hpn = o_sqrt(a);
            rn = o_sqrt(b);
            tpn = o_sqrt(c);
            dh = hpn > 1e-12f ? hpn : 1e-12f;
            dr = rn > 1e-12f ? rn : 1e-12f;
            dt = tpn > 1e-12f ? tpn : 1e-12f;
        }
        float s = 0.f;
        for (int64_t i = 0; i < d; ++i) {
            const float x = v(i);
            s += p == 1 ? fabsf(x) : x * x;
        }
        sc = p == 1 ? s : o_sqrt(s);
    }

    // d score / d v scaled by ds (sign(0) = 0; the L2 gradient is 0 at a zero norm)
    __device__ __forceinline__ float gv(int64_t i, float ds, float q) const {
        const float x = v(i);
        if (p == 1) return x > 0.f ? ds : (x < 0.f ? -ds : 0.f);
        return sc == 0.f ? 0.f : x * q;
    }

    // gradient rows of this slot (oracle.c slot_backward): oh / ot / orr / ow = the batch_h, batch_t,
    // batch_r and norm_vector(batch_r) lookups' rows
    __device__ void backward(float ds, float *oh, float *ot, float *orr, float *ow) const {
        const float q = p == 1 ? 0.f : o_div(ds, sc);
        if (nf) {
            // F.normalize backward: c = (g . x) / (n n); out = (g - x c) / n  (n <= eps: g / eps)
            float sh = 0.f, sr = 0.f, st = 0.f;
            for (int64_t i = 0; i < d; ++i) {
                const float g = gv(i, ds, q);
                sh += g * hp(i);
                sr += g * re[i];
                st += (-g) * tp(i);
            }
            const float ch = o_div(sh, hpn * hpn), cr = o_div(sr, rn * rn), ct = o_div(st, tpn * tpn);
            for (int64_t i = 0; i < d; ++i) {
                const float g = gv(i, ds, q), mg = -g;
                oh[i] = hpn > 1e-12f ? o_div(g - hp(i) * ch, hpn) : o_div(g, 1e-12f);
                orr[i] = rn > 1e-12f ? o_div(g - re[i] * cr, rn) : o_div(g, 1e-12f);
                ot[i] = tpn > 1e-12f ? o_div(mg - tp(i) * ct, tpn) : o_div(mg, 1e-12f);
            }
        } else {
            for (int64_t i = 0; i < d; ++i) {
                const float g = gv(i, ds, q);
                oh[i] = g;
                orr[i] = g;
                ot[i] = -g;
            }
        }
        if (model) {
            // e_perp = e - (e . n) n: g_e = g_p - n (n . g_p); per _transfer call g_n = -((e . n) g_p + (n . g_p) e)
            // through its own F.normalize(norm) backward, the two calls' rows added
            float a = 0.f, b = 0.f;
            for (int64_t i = 0; i < d; ++i) {
                const float n = nw(i);
                a += n * oh[i];
                b += n * ot[i];
            }
            const float nga = a, ngc = b;
            float c1 = 0.f, c2 = 0.f;
            for (int64_t i = 0; i < d; ++i) {
                const float g1 = -(hdot * oh[i] + nga * he[i]);
                const float g2 = -(tdot * ot[i] + ngc * te[i]);
                c1 += g1 * we[i];
                c2 += g2 * we[i];
            }
            c1 = o_div(c1, wn * wn);
            c2 = o_div(c2, wn * wn);
            for (int64_t i = 0; i < d; ++i) {
                const float g1 = -(hdot * oh[i] + nga * he[i]);
                const float g2 = -(tdot * ot[i] + ngc * te[i]);
                const float x1 = wn > 1e-12f ? o_div(g1 - we[i] * c1, wn) : o_div(g1, 1e-12f);
                const float x2 = wn > 1e-12f ? o_div(g2 - we[i] * c2, wn) : o_div(g2, 1e-12f);
                ow[i] = x1 + x2;
                const float n = nw(i);
                oh[i] = oh[i] - n * nga;
                ot[i] = ot[i] - n * ngc;
            }
        }
    }
};

__device__ __forceinline__ void o_update(int opt, float lr, float *w, float *acc, float g) {
    if (opt == 0) {
        *w = *w + (-lr) * g;
    } else {
        const float a = *acc + g * g;
        *acc = a;
        *w = *w + o_div((-lr) * g, o_sqrt(a) + 1e-10f);
    }
}

// MarginLoss coefficient of one (positive, negative) pair: 1/(bs neg) where p - n > -m, half at a tie
__device__ __forceinline__ float o_coef(float ps, float ns, float m, float inv) {
    const float a = ps - ns;
    return a > -m ? inv : (a == -m ? inv / 2 : 0.f);
}

// ------------------------------------------------------------------ single model, grid-wide -----
__global__ void k_ord_score(OrderedStep S) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S.seq) return;
    const int64_t d = S.dim;
    OSlot o{S.ent + S.h[s] * d, S.ent + S.t[s] * d, S.rel + S.r[s] * d,
            S.model ? S.normv + S.r[s] * d : nullptr, d, S.model, S.p_norm, S.norm_flag};
    o.forward();
    S.score[s] = o.sc;
}

// thread i < bs: the coefficients of positive i (ds[i] = sum over k in order, ds[negative] = -c);
// block 0's last wave: the loss, summed in (positive, negative) order in double by one lane
__global__ void k_ord_coef(OrderedStep S, float *loss, int assign) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const float m = S.margin, inv = 1.0f / (float)(S.bs * S.neg);
    if (i < S.bs) {
        float acc = 0.f;
        for (int64_t k = 0; k < S.neg; ++k) {
            const int64_t o = S.bs + k * S.bs + i;
            const float c = o_coef(S.score[i], S.score[o], m, inv);
            acc += c;
            S.ds[o] = 0.f - c;
        }
        S.ds[i] = acc;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && loss) {
        double l = 0.0;
        for (int64_t b = 0; b < S.bs; ++b)
            for (int64_t k = 0; k < S.neg; ++k) {
                const float a = S.score[b] - S.score[S.bs + k * S.bs + b];
                l += (double)(a > -m ? a : -m);
            }
        const float v = (float)(l / (double)(S.bs * S.neg)) + m;
        *loss = assign ? v : *loss + v;
    }
}

__global__ void k_ord_grad(OrderedStep S) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S.seq) return;
    const float ds = S.ds[s];
    if (ds == 0.f) return;
    const int64_t d = S.dim;
    OSlot o{S.ent + S.h[s] * d, S.ent + S.t[s] * d, S.rel + S.r[s] * d,
            S.model ? S.normv + S.r[s] * d : nullptr, d, S.model, S.p_norm, S.norm_flag};
    o.forward();
    o.backward(ds, S.gh + s * d, S.gt + s * d, S.gr + s * d, S.model ? S.gw + s * d : nullptr);
}

// One workgroup per table row (entities [0, E), relations [E, E+R), norm_vector rows [E+R, E+2R)): the
// slots of the row's lookups found in slot order (chunks of NT slots, compacted in order through a
// per-wave ballot), their rows summed in that order per element, then the optimizer.
template <int NT>
__global__ __launch_bounds__(NT) void k_ord_reduce(OrderedStep S) {
    constexpr int NW = NT / 64, MAXE = 8;   // elements per thread: dim <= NT * MAXE
    __shared__ int32_t la[NT], lb[NT];
    __shared__ int wa[NW], wb[NW];
    const int64_t q = blockIdx.x;
    const int64_t E = S.ent_total, R = S.rel_total, d = S.dim;
    const int table = q < E ? 0 : (q < E + R ? 1 : 2);
    const int64_t row = table == 0 ? q : (table == 1 ? q - E : q - E - R);
    const int64_t *ka = table == 0 ? S.h : S.r;
    const int64_t *kb = table == 0 ? S.t : nullptr;
    const float *ga = table == 0 ? S.gh : (table == 1 ? S.gr : S.gw);
    const float *gb = S.gt;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    float acca[MAXE], accb[MAXE];
#pragma unroll
    for (int e = 0; e < MAXE; ++e) acca[e] = accb[e] = 0.f;
    int64_t tota = 0, totb = 0;
    for (int64_t c0 = 0; c0 < S.seq; c0 += NT) {
        const int64_t s = c0 + tid;
        const bool live = s < S.seq && S.ds[s] != 0.f;
        const bool ma = live && ka[s] == row;
        const bool mb = live && kb && kb[s] == row;
        const uint64_t ba = __ballot(ma), bb = __ballot(mb);
        if (lane == 0) {
            wa[wv] = __popcll(ba);
            wb[wv] = __popcll(bb);
        }
        __syncthreads();
        int oa = 0, ob = 0, na = 0, nb = 0;
        for (int w = 0; w < NW; ++w) {
            if (w < wv) {
                oa += wa[w];
                ob += wb[w];
            }
            na += wa[w];
            nb += wb[w];
        }
        const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
        if (ma) la[oa + __popcll(ba & below)] = (int32_t)(s - c0);
        if (mb) lb[ob + __popcll(bb & below)] = (int32_t)(s - c0);
        __syncthreads();
#pragma unroll
        for (int e = 0; e < MAXE; ++e) {
            const int64_t i = tid + (int64_t)e * NT;
            if (i < d) {
                for (int k = 0; k < na; ++k) acca[e] += ga[(c0 + la[k]) * d + i];
                for (int k = 0; k < nb; ++k) accb[e] += gb[(c0 + lb[k]) * d + i];
            }
        }
        tota += na;
        totb += nb;
        __syncthreads();
    }
    if (tota + totb == 0) return;
    float *w = table == 0 ? S.ent : (table == 1 ? S.rel : S.normv);
    float *acc = table == 0 ? S.ent_acc : (table == 1 ? S.rel_acc : S.norm_acc);
#pragma unroll
    for (int e = 0; e < MAXE; ++e) {
        const int64_t i = tid + (int64_t)e * NT;
        if (i < d) {
            const float g = totb ? acca[e] + accb[e] : acca[e];
            o_update(S.opt, S.lr, w + row * d + i, S.opt ? acc + row * d + i : nullptr, g);
        }
    }
}

// ------------------------------------------------------------------ universes, one workgroup each ---
// LDS of a universe workgroup (host-sized for the set's largest universe, int32 units):
//   bh, bt, br [seq] | score, ds [seq] (float) | entity entries (key << 1 | lookup, slot) sorted [2 seq]
//   | relation entries sorted [seq] | row runs [4 seq][3] (first entry, end entry, table << 30 | key)
struct OUniShared {
    int32_t *bh, *bt, *br;
    float *score, *ds;
    int32_t *ent_sorted, *rel_sorted;   // slots, sorted by (key, lookup, slot)
    int32_t *ent_key, *rel_key;         // the sorted entries' (key << 1 | lookup) / key
    int32_t *runs;                      // [3 * nruns]: first entry, end entry, table << 30 | key
    int *nruns, *nent, *nrel;
    uint64_t *states;
    double *epoch_loss;
};

template <int NT>
__device__ void universe_run_ordered(const UniverseDev &U, int model, int p, int nf, int opt, int64_t neg, int bern,
                                     int filter, const OUniShared &S) {
    const int tid = threadIdx.x;
    const int64_t bs = U.bs, threads = U.threads, d = U.dim;
    const int64_t seq = bs * (1 + neg), dpp = 1 + 2 * neg;
    const DeviceGraph &g = U.g;
    const float m = U.margin, inv = 1.0f / (float)(bs * neg);
    float *gh = U.ord, *gt = gh + seq * d, *gr = gt + seq * d, *gw = gr + seq * d;
    if (tid < threads) S.states[tid] = U.states[tid];
    if (tid == 0) *S.epoch_loss = 0.0;
    __syncthreads();
    for (int64_t epoch = 0; epoch < U.epochs; ++epoch) {
        for (int64_t step = 0; step < U.nbatches; ++step) {
            // ---- sampling() call: positives and negatives in the reference layout (Base.cpp:185-264)
            for (int64_t b = tid; b < bs; b += NT) {
                const PosDraw pd = draw_positive(g, S.states, threads, bs, b, dpp);
                S.bh[b] = (int32_t)pd.h; S.br[b] = (int32_t)pd.r; S.bt[b] = (int32_t)pd.t;
                for (int64_t k = 0; k < neg; ++k) {
                    int side;
                    const int64_t e = draw_negative(g, pd, k, bern, filter, &side);
                    const int64_t o = (k + 1) * bs + b;
                    S.bh[o] = (int32_t)(side ? pd.h : e);
                    S.bt[o] = (int32_t)(side ? e : pd.t);
                    S.br[o] = (int32_t)pd.r;
                }
            }
            __syncthreads();
            if (tid < threads) {
                const int64_t per = bs % threads == 0 ? bs / threads : bs / threads + 1;
                int64_t len = bs - tid * per;
                len = len < 0 ? 0 : (len > per ? per : len);
                S.states[tid] = lcg_jump(S.states[tid], (uint64_t)(len * dpp));
            }
            // ---- scores
            for (int64_t s = tid; s < seq; s += NT) {
                OSlot o{U.ent + S.bh[s] * d, U.ent + S.bt[s] * d, U.rel + S.br[s] * d,
                        model ? U.normv + S.br[s] * d : nullptr, d, model, p, nf};
                o.forward();
                S.score[s] = o.sc;
            }
            __syncthreads();
            // ---- coefficients; the loss (one lane, in order, while the others go on)
            for (int64_t i = tid; i < bs; i += NT) {
                float acc = 0.f;
                for (int64_t k = 0; k < neg; ++k) {
                    const int64_t o = bs + k * bs + i;
                    const float c = o_coef(S.score[i], S.score[o], m, inv);
                    acc += c;
                    S.ds[o] = 0.f - c;
                }
                S.ds[i] = acc;
            }
            if (tid == 0) {
                double l = 0.0;
                for (int64_t b = 0; b < bs; ++b)
                    for (int64_t k = 0; k < neg; ++k) {
                        const float a = S.score[b] - S.score[bs + k * bs + b];
                        l += (double)(a > -m ? a : -m);
                    }
                *S.epoch_loss += (double)((float)(l / (double)(bs * neg)) + m);
            }
            __syncthreads();
            // ---- per-slot gradient rows
            for (int64_t s = tid; s < seq; s += NT) {
                const float ds = S.ds[s];
                if (ds == 0.f) continue;
                OSlot o{U.ent + S.bh[s] * d, U.ent + S.bt[s] * d, U.rel + S.br[s] * d,
                        model ? U.normv + S.br[s] * d : nullptr, d, model, p, nf};
                o.forward();
                o.backward(ds, gh + s * d, gt + s * d, gr + s * d, model ? gw + s * d : nullptr);
            }
            // ---- entries sorted by (key, lookup, slot): position = number of smaller live entries
            //      (entity entries: lookup 0 = batch_h, 1 = batch_t; relation entries: batch_r)
            if (tid == 0) *S.nruns = 0;
            for (int64_t x = tid; x < 3 * seq; x += NT) {
                const bool ent = x < 2 * seq;
                const int64_t s = ent ? (x < seq ? x : x - seq) : x - 2 * seq;
                if (S.ds[s] == 0.f) continue;
                const int look = ent && x >= seq ? 1 : 0;
                const int32_t key = ent ? ((look ? S.bt[s] : S.bh[s]) << 1 | look) : S.br[s];
                int32_t pos = 0;
                for (int64_t y = 0; y < seq; ++y) {
                    if (S.ds[y] == 0.f) continue;
                    if (ent) {
                        const int32_t k0 = S.bh[y] << 1, k1 = S.bt[y] << 1 | 1;
                        pos += (k0 < key || (k0 == key && y < s)) + (k1 < key || (k1 == key && y < s));
                    } else {
                        const int32_t k = S.br[y];
                        pos += k < key || (k == key && y < s);
                    }
                }
                if (ent) {
                    S.ent_sorted[pos] = (int32_t)s;
                    S.ent_key[pos] = key;
                } else {
                    S.rel_sorted[pos] = (int32_t)s;
                    S.rel_key[pos] = key;
                }
            }
            if (tid == 0) {
                int n = 0;
                for (int64_t s = 0; s < seq; ++s) n += S.ds[s] != 0.f;
                *S.nent = 2 * n;
                *S.nrel = n;
            }
            __syncthreads();   // (also orders the gradient rows' stores before the reduce reads them)
            // ---- row runs: entity rows (both lookups of a key), relation rows, norm_vector rows
            const int nent = *S.nent, nrel = *S.nrel;
            for (int x = tid; x < nent + nrel; x += NT) {
                const bool ent = x < nent;
                const int j = ent ? x : x - nent;
                const int32_t *key = ent ? S.ent_key : S.rel_key;
                const int n = ent ? nent : nrel;
                const int32_t k = ent ? key[j] >> 1 : key[j];
                const bool head = j == 0 || (ent ? key[j - 1] >> 1 : key[j - 1]) != k;
                if (!head) continue;
                int e = j + 1;
                while (e < n && (ent ? key[e] >> 1 : key[e]) == k) ++e;
                const int tables = ent ? 1 : (model ? 2 : 1);
                for (int tb = 0; tb < tables; ++tb) {
                    const int r = atomicAdd(S.nruns, 1);
                    S.runs[3 * r] = j;
                    S.runs[3 * r + 1] = e;
                    S.runs[3 * r + 2] = (ent ? 0 : 1 + tb) << 30 | k;
                }
            }
            __syncthreads();
            // ---- per (row, element): the lookups' rows in slot order, the entity lookups added, update
            const int64_t items = (int64_t)*S.nruns * d;
            for (int64_t f = tid; f < items; f += NT) {
                const int r = (int)(f / d);
                const int64_t i = f - (int64_t)r * d;
                const int j0 = S.runs[3 * r], j1 = S.runs[3 * r + 1];
                const int tb = S.runs[3 * r + 2] >> 30;
                const int64_t row = S.runs[3 * r + 2] & ((1 << 30) - 1);
                float a = 0.f, b = 0.f;
                int nb = 0;
                if (tb == 0) {
                    for (int j = j0; j < j1; ++j) {
                        const int64_t s = S.ent_sorted[j];
                        if (S.ent_key[j] & 1) {
                            b += gt[s * d + i];
                            ++nb;
                        } else {
                            a += gh[s * d + i];
                        }
                    }
                } else {
                    const float *src = tb == 1 ? gr : gw;
                    for (int j = j0; j < j1; ++j) a += src[(int64_t)S.rel_sorted[j] * d + i];
                }
                const bool only_b = tb == 0 && nb == j1 - j0;
                const float gsum = only_b ? b : (nb ? a + b : a);
                float *w = tb == 0 ? U.ent : (tb == 1 ? U.rel : U.normv);
                float *acc = tb == 0 ? U.ent_acc : (tb == 1 ? U.rel_acc : U.norm_acc);
                o_update(opt, U.lr, w + row * d + i, opt ? acc + row * d + i : nullptr, gsum);
            }
            __syncthreads();   // the next step reads the updated tables
        }
        if (tid == 0) {
            if (U.losses) U.losses[epoch] = (float)*S.epoch_loss;
            *S.epoch_loss = 0.0;
        }
    }
    if (tid < threads) U.states[tid] = S.states[tid];
}

template <int NT>
__global__ __launch_bounds__(NT) void k_universes_ordered(const UniverseDev *__restrict__ us, int64_t n,
                                                          int *__restrict__ next_universe, int model, int p, int nf,
                                                          int opt, int64_t neg, int bern, int filter, int64_t max_seq) {
    extern __shared__ int32_t s_dyn[];
    __shared__ uint64_t s_states[64];
    __shared__ double s_loss;
    __shared__ int s_u, s_nruns, s_nent, s_nrel;
    OUniShared S;
    int32_t *q = s_dyn;
    S.bh = q; q += max_seq;
    S.bt = q; q += max_seq;
    S.br = q; q += max_seq;
    S.score = reinterpret_cast<float *>(q); q += max_seq;
    S.ds = reinterpret_cast<float *>(q); q += max_seq;
    S.ent_sorted = q; q += 2 * max_seq;
    S.ent_key = q; q += 2 * max_seq;
    S.rel_sorted = q; q += max_seq;
    S.rel_key = q; q += max_seq;
    S.runs = q;
    S.nruns = &s_nruns; S.nent = &s_nent; S.nrel = &s_nrel;
    S.states = s_states;
    S.epoch_loss = &s_loss;
    for (;;) {
        if (threadIdx.x == 0) s_u = atomicAdd(next_universe, 1);
        __syncthreads();
        const int64_t u = s_u;
        __syncthreads();
        if (u >= n) break;
        universe_run_ordered<NT>(us[u], model, p, nf, opt, neg, bern, filter, S);
        __syncthreads();
    }
}

}  // namespace dev

// ------------------------------------------------------------------ launchers --------------------
hipError_t launch_ordered_step(const OrderedStep &S, float *loss, int assign, hipStream_t st) {
    if (S.seq <= 0) return hipSuccess;
    const unsigned blocks = (unsigned)((S.seq + 63) / 64);
    hipLaunchKernelGGL(dev::k_ord_score, dim3(blocks), dim3(64), 0, st, S);
    hipLaunchKernelGGL(dev::k_ord_coef, dim3((unsigned)((S.bs + 255) / 256)), dim3(256), 0, st, S, loss, assign);
    hipLaunchKernelGGL(dev::k_ord_grad, dim3(blocks), dim3(64), 0, st, S);
    const int64_t rows = S.ent_total + S.rel_total * (S.model ? 2 : 1);
    hipLaunchKernelGGL(dev::k_ord_reduce<256>, dim3((unsigned)rows), dim3(256), 0, st, S);
    return hipGetLastError();
}

bool ordered_dim_supported(int64_t dim) { return dim > 0 && dim <= 256 * 8; }

int64_t ordered_universe_lds_bytes(int64_t max_seq) { return 4 * (11 * max_seq + 12 * max_seq); }

hipError_t ordered_universe_static_lds(size_t *bytes) {
    hipFuncAttributes a{};
    const hipError_t e = hipFuncGetAttributes(&a, reinterpret_cast<const void *>(dev::k_universes_ordered<256>));
    if (e == hipSuccess) *bytes = a.sharedSizeBytes;
    return e;
}

hipError_t launch_universes_ordered(const UniverseDev *d_us, int64_t n, int *counter, int64_t cus, int model,
                                    int p_norm, int norm_flag, int opt, int64_t neg, int bern, int filter,
                                    int64_t max_seq, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    constexpr int NT = 256;
    auto kern = dev::k_universes_ordered<NT>;
    const int64_t lds = ordered_universe_lds_bytes(max_seq);
    if (lds > (64 << 10)) {
        const hipError_t e =
            hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    int64_t grid = cus * 2;
    if (grid > n) grid = n;
    hipError_t e = hipMemsetAsync(counter, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), (size_t)lds, st, d_us, n, counter, model, p_norm,
                       norm_flag, opt, neg, bern, filter, max_seq);
    return hipGetLastError();
}

}  // namespace pt
