// Fused TransE training step + sparse optimizer apply on a counting-sort batch: the C2 hot path in ONE
// launch per step (step.hip's k_step_csr and apply.hip's k_apply_buf in one kernel).
//
// Why: as two launches, the step's corrupted-entity gradient rows (contribution rows, 40 MB per C2 step)
// are written by k_step_csr and read back by k_apply_buf only after the whole step kernel has drained,
// and the apply's ~15k row updates run as a second, latency-bound pass. Here every table row is updated
// by the wave that delivers its LAST gradient contribution of the step, inside the step kernel, while
// the rest of the chip still computes - no second pass, no launch boundary.
//
// Arrivals. Each entity row e receives, per step, one contribution row per negative slot that corrupted
// to e (its counting-sort bucket: start[e] .. start[e+1]) plus one arrival per use of e as a positive's h
// or t (the positive's gradient rows go to padded gradient rows by memory-side float atomics); relation
// row r one arrival per positive with relation r. The sampler counts the positives' uses (CsrWork::uses),
// so every row's arrival count is known before the step. A wave arrives - one agent-scope atomic add per
// row - only after the data it contributes is complete: its contribution rows stored write-through (sc1,
// whole 128-B lines: rows are padded to a multiple of 32 floats) or its atomics done, and an
// `s_waitcnt vmcnt(0)`; the add whose returned count completes the row's total makes that wave the row's
// last arriver (MI355X_MICROARCH.md, visibility table row 1: counter add after every storing wave's wait,
// the consumer told by the value its add returned, every load of the handed-off bytes an sc1 load). The
// last arriver re-zeroes the row's arrival word, loads the row's gradient rows (sc1) and contributions in
// bucket order, applies the normalize Jacobian of the pre-step row and SGD / Adagrad - the same operations
// in the same order as k_apply_buf - and zeroes the row's gradient row for the next step. A row is only
// written after every reader of its pre-step value in this step has arrived (each reader of a row is one
// of its arrivals), so no wave can see a half-updated table.
//
// Measured (r04, driver-shaped C2, same boxes): correct - equal to the pair to 4e-9 after a step, every parity
// test green - but SLOWER: 35.7 us per step for this kernel against 20.9 + 11.9 us for k_step_csr + k_apply_buf
// (the line: 40.1-42.0 vs 36.2-36.9 us/step). Each wave's tail gains three dependent memory round trips (drain,
// arrival add, the row's loads) and at 115 VGPRs the 8,000 waves of a step run in two occupancy rounds, so
// the tails add up instead of overlapping; two waves per positive (one round): 46 us; 8 waves per SIMD (64
// VGPRs, spilling): 62 us. It stays an opt-in mode (pt_trainer_set_step_apply); the pair is the default.
//
// Semantics as step.hip / apply.hip: sampler = Base.cpp:185-310 + Corrupt.h:9-105; forward TransE.py:46-74;
// loss MarginLoss.py:24-28; update torch.optim.SGD / Adagrad as built in Trainer.py:62-88.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "tuning.h"
#include "device.h"
#include "kernels.h"
#include "step_apply.h"

namespace pt {
namespace dev {

// row arrival words: low 32 bits count arrivals, each arrival that carried a gradient row adds kCarried
constexpr uint64_t kCarried = uint64_t(1) << 32;

__device__ __forceinline__ uint64_t arrive_add(uint64_t *p, uint64_t v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void arrive_reset(uint64_t *p) {
    __hip_atomic_store(p, uint64_t(0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every vector-memory operation this wave issued has completed (its stores and atomics are performed)
__device__ __forceinline__ void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// raw-buffer row loads / stores with the sc1 cache policy (aux 16): loads bypass this CU's L1, stores
// write through to memory and leave no copy in the XCD's L2
template <int G, int VEC, int KCH>
__device__ __forceinline__ void bload_sc1(V<G, VEC, KCH> &o, __amdgpu_buffer_rsrc_t rs, uint32_t row_bytes, int D,
                                          int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        const uint32_t off = c * VEC < D ? row_bytes + (uint32_t)(c * VEC * 4) : kOob;
        const pt_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
        o.x[k * 4 + 0] = __uint_as_float(v.x); o.x[k * 4 + 1] = __uint_as_float(v.y);
        o.x[k * 4 + 2] = __uint_as_float(v.z); o.x[k * 4 + 3] = __uint_as_float(v.w);
    }
}
// a whole padded row (dp floats): lanes past the row's D floats store zeros, so every 128-B line of the
// row is written by one store instruction
template <int G, int VEC, int KCH>
__device__ __forceinline__ void bstore_row_sc1(const V<G, VEC, KCH> &o, __amdgpu_buffer_rsrc_t rs, uint32_t row_bytes,
                                               int D, int dp, int lane) {
#pragma unroll
    for (int k = 0; k < KCH; ++k) {
        const int c = k * G + lane;
        const bool in = c * VEC < D;
        const uint32_t off = c * VEC < dp ? row_bytes + (uint32_t)(c * VEC * 4) : kOob;
        const pt_u32x4 v = {in ? __float_as_uint(o.x[k * 4 + 0]) : 0u, in ? __float_as_uint(o.x[k * 4 + 1]) : 0u,
                            in ? __float_as_uint(o.x[k * 4 + 2]) : 0u, in ? __float_as_uint(o.x[k * 4 + 3]) : 0u};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
    }
}

// The last arriver's update of one table row (k_apply_buf's operations in its order): g = the row's
// gradient row (if an arrival carried one) + its bucket's contribution rows in counting-sort order;
// normalize Jacobian of the pre-step row (jac); SGD / Adagrad; the gradient row re-zeroed.
template <int KCH>
__device__ __forceinline__ void apply_row(const StepParams &P, float *tab, float *acc, int64_t rows, float *grad,
                                          const float *contrib, int64_t row, int c0, int c1, bool carried, bool jac,
                                          int D, int dp, int lane) {
    using Vec = V<64, 4, KCH>;
    const uint32_t rowb = (uint32_t)D * 4u, prow = (uint32_t)dp * 4u;
    const auto t_rs = make_rsrc(tab, (uint32_t)rows * rowb);
    const auto g_rs = make_rsrc(grad, (uint32_t)rows * prow);
    Vec x, a, g;
    bload(x, t_rs, (uint32_t)row * rowb, D, lane);
    if (P.opt != 0) bload(a, make_rsrc(acc, (uint32_t)rows * rowb), (uint32_t)row * rowb, D, lane);
    bload_sc1(g, g_rs, carried ? (uint32_t)row * prow : kOob, D, lane);
    if (c1 > c0) {
        const auto c_rs = make_rsrc(contrib, 0x7fffffffu);
        for (int j = c0; j < c1; j += 8) {
            Vec c[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) bload_sc1(c[u], c_rs, j + u < c1 ? (uint32_t)(j + u) * prow : kOob, D, lane);
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int i = 0; i < Vec::N; ++i) g.x[i] += c[u].x[i];
        }
    }
    Vec gg;
    if (jac) {
        const float n = sqrtf(vdot(x, x));
        vnormalize_bwd(x, n, g, gg);
    } else {
        gg = g;
    }
    if (P.opt == 0) {
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) x.x[i] = x.x[i] + (-P.lr) * gg.x[i];
    } else {
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            a.x[i] = a.x[i] + gg.x[i] * gg.x[i];
            x.x[i] = x.x[i] + (-P.lr) * gg.x[i] / (sqrtf(a.x[i]) + 1e-10f);
        }
        bstore(a, make_rsrc(acc, (uint32_t)rows * rowb), (uint32_t)row * rowb, D, lane);
    }
    bstore(x, t_rs, (uint32_t)row * rowb, D, lane);
    if (carried) {
        Vec z;
        vzero(z);
        bstore(z, g_rs, (uint32_t)row * prow, D, lane);
    }
}

// One positive per workgroup of S waves (lane group = wave, float4 lanes, KCH chunks per lane); wave s
// takes negatives [s * nper, (s + 1) * nper) in windows of 64 (one record per lane), their rows double-
// buffered NCH at a time as in k_step_csr. A window's slots arrive once its contribution rows are stored;
// the last window's after the sub-groups' partials have met in LDS, together with the positive's h / t / r
// arrivals (wave 0, after its gradient-row atomics).
template <int KCH, int NCH, int S, int PN>
__global__ __launch_bounds__(S * 64) void k_step_apply(StepParams P, CsrWork cw, FusedRows fr) {
    constexpr int G = 64, VEC = 4;
    using Vec = V<G, VEC, KCH>;
    constexpr int RW = KCH * G * VEC;
    __shared__ float red[S > 1 ? S * 2 * RW + 2 * S : 1];
    __shared__ float trb[3 * RW];   // positive-row gradients, transposed for 256-B atomics
    const int lane = (int)threadIdx.x & 63;
    const int sub = (int)threadIdx.x >> 6;
    const int64_t b = blockIdx.x;
    const int D = (int)P.dim, dp = fr.dp;
    const uint32_t rowb = (uint32_t)D * 4u, prow = (uint32_t)dp * 4u;
    const int neg = (int)P.neg;
    constexpr int p = PN;
    const bool nf = P.norm_flag != 0;
    const float m = P.margin, inv = P.inv_count;
    const int64_t E = P.ent_total;
    const int nper = (neg + S - 1) / S;
    const int k_lo = sub * nper < neg ? sub * nper : neg;
    const int k_hi = k_lo + nper < neg ? k_lo + nper : neg;
    const auto ent_rs = make_rsrc(P.ent, (uint32_t)E * rowb);
    const auto rel_rs = make_rsrc(P.rel, (uint32_t)P.rel_total * rowb);
    const auto con_rs = make_rsrc(cw.contrib, (uint32_t)(P.batch_size * neg) * prow);
    const int4 q = cw.pos[b];
    const int32_t hp = uni<G>(q.x), rp = uni<G>(q.y), tp = uni<G>(q.z);
    const int32_t *nrec = cw.neg + b * neg;
    const int32_t *ndst = cw.off + b * neg;
    // this lane's slot of the current window [wlo, whi): record, destination row, its entity's bucket and uses
    int wlo = k_lo, whi = k_hi - k_lo < G ? k_hi : k_lo + G;
    int32_t rec = 0, dst = 0, s0 = 0, s1 = 0, pu = 0;
    auto fetch_window = [&]() {
        rec = dst = s0 = s1 = pu = 0;
        if (wlo + lane < whi) {
            rec = nrec[wlo + lane];
            dst = ndst[wlo + lane];
            const int32_t e = rec >> 1;
            s0 = cw.start[e];
            s1 = cw.start[e + 1];
            pu = cw.uses[e];
            if (cw.rank_only) dst += s0;   // rank in the bucket -> destination row
        }
    };
    // the window's slots arrive: every row whose count this completes is updated here, by this wave
    auto arrive_window = [&]() {
        drain_vmem();
        const bool mine = wlo + lane < whi;
        const int32_t e = rec >> 1;
        uint64_t now = 0;
        if (mine) now = arrive_add(fr.arrive + e, 1) + 1;
        const bool last = mine && (uint32_t)now == (uint32_t)(s1 - s0 + pu);
        if (last) arrive_reset(fr.arrive + e);
        uint64_t mask = __ballot(last);
        while (mask) {
            const int j = __builtin_ctzll(mask);
            mask &= mask - 1;
            const int32_t ej = __builtin_amdgcn_readlane(e, j);
            const int32_t c0 = __builtin_amdgcn_readlane(s0, j), c1 = __builtin_amdgcn_readlane(s1, j);
            const bool carried = __builtin_amdgcn_readlane((int32_t)(now >> 32), j) != 0;
            apply_row<KCH>(P, P.ent, P.ent_acc, E, fr.gent, cw.contrib, ej, c0, c1, carried, nf, D, dp, lane);
        }
    };
    fetch_window();
    // the positive's own rows: h, t (entity rows: their buckets and uses) and r, on lanes 0, 1, 2
    int64_t prow_id = 0;
    int32_t ps0 = 0, ps1 = 0, ppu = 0;
    if (sub == 0 && lane < 3) {
        prow_id = lane == 0 ? hp : (lane == 1 ? tp : cw.rel_base + rp);
        if (lane < 2) {
            ps0 = cw.start[prow_id];
            ps1 = cw.start[prow_id + 1];
        }
        ppu = cw.uses[prow_id];
    }
    Vec At, Ah, rh, th, bt;
    vzero(At); vzero(Ah);
    float csum = 0.f, lsum = 0.f, ps = 0.f;
    {
        Vec H, T, Rr;
        bload(H, ent_rs, (uint32_t)hp * rowb, D, lane);
        bload(T, ent_rs, (uint32_t)tp * rowb, D, lane);
        bload(Rr, rel_rs, (uint32_t)rp * rowb, D, lane);
        // every chunk issues exactly NCH row loads (past the window end: the window's last row again)
        Vec EA[NCH], EB[NCH];
        auto load_chunk = [&](Vec(&X)[NCH], int k0) {
#pragma unroll
            for (int u = 0; u < NCH; ++u) {
                const int kk = k0 + u < whi ? k0 + u : whi - 1;
                const uint32_t e = (uint32_t)(__builtin_amdgcn_readlane(rec, kk - wlo) >> 1);
                bload(X[u], ent_rs, e * rowb, D, lane);
            }
        };
        if (wlo < whi) load_chunk(EA, wlo);
        Vec hh;
        if (nf) {
            vnormalize<true>(H, hh);
            vnormalize<true>(Rr, rh);
            vnormalize<true>(T, th);
        } else {
            hh = H; rh = Rr; th = T;
        }
        Vec vpos;
#pragma unroll
        for (int i = 0; i < Vec::N; ++i) {
            bt.x[i] = hh.x[i] + rh.x[i];
            vpos.x[i] = bt.x[i] - th.x[i];
        }
        ps = vpnorm<true>(vpos, p);
        auto process = [&](Vec(&X)[NCH], int k0) {
#pragma unroll
            for (int u = 0; u < NCH; ++u) {
                if (k0 + u < whi) {
                    const int32_t r = __builtin_amdgcn_readlane(rec, k0 + u - wlo);
                    const int32_t di = __builtin_amdgcn_readlane(dst, k0 + u - wlo);
                    const bool tail_side = r & 1;
                    Vec eh, vk, gs;
                    if (nf) vnormalize<true>(X[u], eh); else eh = X[u];
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
                    // slot gradient d loss / d e-hat (zeros for an inactive pair: the slot must be defined)
                    vpnorm_bwd<true>(vk, ns, p, tail_side ? c : -c, gs);
                    bstore_row_sc1(gs, con_rs, (uint32_t)di * prow, D, dp, lane);
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
        for (;;) {
            for (int c0 = wlo; c0 < whi;) {
                if (c0 + NCH < whi) load_chunk(EB, c0 + NCH);
                process(EA, c0);
                c0 += NCH;
                if (c0 >= whi) break;
                if (c0 + NCH < whi) load_chunk(EA, c0 + NCH);
                process(EB, c0);
                c0 += NCH;
            }
            if (whi >= k_hi) break;
            arrive_window();
            wlo = whi;
            whi = k_hi - wlo < G ? k_hi : wlo + G;
            fetch_window();
            load_chunk(EA, wlo);
        }
    }
    if constexpr (S > 1) {
        // the sub-groups' partials meet in LDS; wave 0 sums them in a fixed order
        float *mr = red + sub * 2 * RW;
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) {
            const int c = ((k / VEC) * G + lane) * VEC + k % VEC;
            mr[c] = At.x[k];
            mr[RW + c] = Ah.x[k];
        }
        float *cs = red + S * 2 * RW;
        if (lane == 0) {
            cs[sub * 2 + 0] = csum;
            cs[sub * 2 + 1] = lsum;
        }
        __syncthreads();
        if (sub != 0) {
            arrive_window();
            return;
        }
        vzero(At); vzero(Ah);
        csum = lsum = 0.f;
        for (int q2 = 0; q2 < S; ++q2) {
            const float *qr = red + q2 * 2 * RW;
#pragma unroll
            for (int k = 0; k < Vec::N; ++k) {
                const int c = ((k / VEC) * G + lane) * VEC + k % VEC;
                At.x[k] += qr[c];
                Ah.x[k] += qr[RW + c];
            }
            csum += cs[q2 * 2 + 0];
            lsum += cs[q2 * 2 + 1];
        }
    }
    if (lane == 0) cw.lpart[b] = lsum;
    const bool carried = uni<G>(csum) != 0.f;
    if (carried) {
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
        // through LDS so lane l adds floats l, l + 64, ... (256 contiguous bytes per atomic instruction)
#pragma unroll
        for (int k = 0; k < Vec::N; ++k) {
            const int c = ((k / VEC) * G + lane) * VEC + k % VEC;
            trb[c] = aR.x[k];
            trb[RW + c] = aH.x[k];
            trb[2 * RW + c] = aT.x[k];
        }
        __builtin_amdgcn_wave_barrier();
        float *gr = fr.grel + (int64_t)rp * dp, *gh = fr.gent + (int64_t)hp * dp, *gt = fr.gent + (int64_t)tp * dp;
#pragma unroll
        for (int k = 0; k < KCH * VEC; ++k) {
            const int c = k * G + lane;
            if (c < D) {
                atomicAdd(gr + c, trb[c]);
                atomicAdd(gh + c, trb[RW + c]);
                atomicAdd(gt + c, trb[2 * RW + c]);
            }
        }
    }
    // the last window's slots and the positive's three rows arrive (one drain for both)
    drain_vmem();
    {
        const bool mine = wlo + lane < whi;
        const int32_t e = rec >> 1;
        uint64_t now = 0, pnow = 0;
        if (mine) now = arrive_add(fr.arrive + e, 1) + 1;
        const uint64_t pinc = carried ? 1 + kCarried : 1;
        if (lane < 3) pnow = arrive_add(fr.arrive + prow_id, pinc) + pinc;
        const bool last = mine && (uint32_t)now == (uint32_t)(s1 - s0 + pu);
        const bool plast = lane < 3 && (uint32_t)pnow == (uint32_t)(ps1 - ps0 + ppu);
        if (last) arrive_reset(fr.arrive + e);
        if (plast) arrive_reset(fr.arrive + prow_id);
        uint64_t mask = __ballot(last);
        while (mask) {
            const int j = __builtin_ctzll(mask);
            mask &= mask - 1;
            const int32_t ej = __builtin_amdgcn_readlane(e, j);
            const int32_t c0 = __builtin_amdgcn_readlane(s0, j), c1 = __builtin_amdgcn_readlane(s1, j);
            const bool cj = __builtin_amdgcn_readlane((int32_t)(now >> 32), j) != 0;
            apply_row<KCH>(P, P.ent, P.ent_acc, E, fr.gent, cw.contrib, ej, c0, c1, cj, nf, D, dp, lane);
        }
        mask = __ballot(plast);
        while (mask) {
            const int j = __builtin_ctzll(mask);
            mask &= mask - 1;
            const bool cj = __builtin_amdgcn_readlane((int32_t)(pnow >> 32), j) != 0;
            if (j < 2) {
                const int32_t ej = j == 0 ? hp : tp;
                const int32_t c0 = __builtin_amdgcn_readlane(ps0, j), c1 = __builtin_amdgcn_readlane(ps1, j);
                apply_row<KCH>(P, P.ent, P.ent_acc, E, fr.gent, cw.contrib, ej, c0, c1, cj, nf, D, dp, lane);
            } else {
                apply_row<KCH>(P, P.rel, P.rel_acc, P.rel_total, fr.grel, nullptr, rp, 0, 0, cj, nf, D, dp, lane);
            }
        }
    }
}

// loss of each call of a chunk from its positives' partials, in apply_block0's order:
// loss = inv_count * sum(lpart) + margin (MarginLoss.py:24-28)
__global__ __launch_bounds__(64) void k_loss_calls(const float *__restrict__ lpart, int64_t bs, float inv_count,
                                                   float margin, float *__restrict__ loss, int assign) {
    const int lane = (int)threadIdx.x;
    const float *lp = lpart + (int64_t)blockIdx.x * bs;
    float s = 0.f;
    for (int64_t i0 = lane; i0 < bs; i0 += 64 * 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = i0 + u * 64 < bs ? lp[i0 + u * 64] : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    s = gsum<64>(s);
    if (lane == 0) {
        const float l = s * inv_count + margin;
        if (assign) loss[blockIdx.x] = l; else loss[blockIdx.x] += l;
    }
}

}  // namespace dev

// ==================================================================== host launchers ===========
int64_t step_apply_row_stride(int64_t dim) { return (dim + 31) & ~int64_t(31); }

bool step_apply_supported(const StepParams &P, int64_t bs, int64_t neg) {
    if (P.model != 0 || P.dim % 4 != 0) return false;
    const int64_t chunks = P.dim / 4;
    if (chunks <= 32 || chunks > 4 * 64) return false;   // one wave per row, 1-4 float4 chunks per lane
    const int64_t dp = step_apply_row_stride(P.dim);
    const int64_t lim = int64_t(1) << 31;
    if (bs * neg * dp * 4 >= lim || P.ent_total * dp * 4 >= lim || (P.ent_total + P.rel_total) * P.dim * 4 >= lim)
        return false;
    return bs * (neg + 2) < (int64_t(1) << 31);
}

hipError_t launch_step_apply(const StepParams &P, const CsrWork &v, const FusedRows &fr, hipStream_t st) {
    if (P.batch_size <= 0) return hipSuccess;
    const int KCH = (int)((P.dim / 4 + 63) / 64);
    int S = 1;
    while (S < 4 && P.neg >= 6 * S * 2) S *= 2;
    const dim3 grid((unsigned)P.batch_size);
#define PT_SA(K_, S_)                                                                                   \
    if (KCH == K_ && S == S_) {                                                                        \
        if (P.p_norm == 1)                                                                             \
            hipLaunchKernelGGL((dev::k_step_apply<K_, 2, S_, 1>), grid, dim3(S_ * 64), 0, st, P, v, fr);   \
        else                                                                                           \
            hipLaunchKernelGGL((dev::k_step_apply<K_, 2, S_, 2>), grid, dim3(S_ * 64), 0, st, P, v, fr);   \
        return hipGetLastError();                                                                      \
    }
    PT_SA(1, 1) PT_SA(1, 2) PT_SA(1, 4) PT_SA(2, 1) PT_SA(2, 2) PT_SA(2, 4)
    PT_SA(3, 1) PT_SA(3, 2) PT_SA(3, 4) PT_SA(4, 1) PT_SA(4, 2) PT_SA(4, 4)
#undef PT_SA
    return hipErrorInvalidValue;
}

hipError_t launch_loss_calls(const float *lpart, int64_t bs, int64_t calls, float inv_count, float margin, float *loss,
                             int assign, hipStream_t st) {
    if (calls <= 0 || !loss) return hipSuccess;
    hipLaunchKernelGGL(dev::k_loss_calls, dim3((unsigned)calls), dim3(64), 0, st, lpart, bs, inv_count, margin, loss,
                       assign);
    return hipGetLastError();
}

}  // namespace pt
