// Team universes: one universe trained by a TEAM of W workgroups on W CUs (TransE, the 1,024-thread row shapes).
//
// A universe's training is a chain of ~epochs x 20 dependent minibatch steps (Parallel_Universe_Config.py:228-258),
// and one workgroup runs it (universes_kern.h). When a GPU holds fewer universes than CUs - the BASELINE PU configs
// at 8 GPUs: C4 128, C3 64, C5 32 universes per GPU on 256 CUs - the set's makespan is its longest chain and most
// CUs idle. A team splits each step of one universe over its members:
//
//   presample  every member draws the same batches into its own LDS (universe_run's Presampler: no exchange);
//   link pass  every member links the step's entity rows to their STATIC contribution slots (slot b * (neg + 2) + k:
//              negative k, then head, then tail of positive b) in its own LDS lists, from the batch alone, and
//              collects the step's rows - the same sets on every member, each member also the rows it owns
//              (entity / relation id mod W);
//   phase A    member m runs positives b = m, m + W, ... (transe_step with ALWAYS: every slot of a positive is
//              written, zero for an inactive pair), relation gradients into its LDS rows, which it then publishes
//              as its partial of each step relation;
//   barrier    (team_barrier)
//   phase B    member m updates the rows it owns: an entity row sums its slots along its list, a relation row the W
//              members' partials in member order; normalize Jacobian of the pre-step row, Adagrad / SGD;
//   barrier.
// Every exchanged byte (contribution rows, relation partials, the universe's table rows and Adagrad state, loss
// partials) is written with sc1 buffer stores, drained (vmcnt(0)) before the arrival atomic, and read with sc1 buffer
// loads: the hand-off form of MI355X_MICROARCH.md ("Inter-workgroup visibility"), correct wherever the members run.
// The counter is monotonic per train call (2 arrivals per member per step, zeroed by the host before the launch).
// Each poll is bounded (team_barrier): a stuck team raises an error word the host checks, it never hangs the GPU.
//
// Team members must be co-resident: the host sizes the launches of a set so that every workgroup of every
// concurrent launch has a CU (pt_universe_set_create), and no workgroup waits on anything but its own team.
#pragma once
#include "universes_kern.h"

namespace pt {
namespace dev {

// all members of a team past the same point: this wave's sc1 stores complete, one agent-scope arrival per member,
// then a poll of the team's counter up to `target` (= members x barriers so far)
// The poll is bounded (about 2^25 sleeps, seconds - a set's whole training takes milliseconds): a member that never
// arrives (a launch whose workgroups were not all resident) raises the team error word instead of hanging the GPU,
// and the host reports the train call as failed.
__device__ __forceinline__ void team_barrier(uint32_t *ctr, uint32_t target, uint32_t *err) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t spin = 0; __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
            if (spin >= (1u << 25)) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

// gradient sink of a team member: entity rows to the positive's static slots (sc1 stores), relation rows into the
// member's LDS gradient rows (its partials)
struct TeamSink {
    __amdgpu_buffer_rsrc_t contrib;
    float *grel;                 // LDS [R][D]
    mutable int slot = 0;
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void ent(int, const V<G, VEC, KCH> &g, int D, int lane) const {
        bstore<G, VEC, KCH, 16>(g, contrib, (uint32_t)(slot++ * D * 4), D, lane);
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void rel(int row, const V<G, VEC, KCH> &g, int D, int lane) const {
        vatomic(g, grel + row * D, D, lane);
    }
    uint64_t *trace = nullptr;   // (transe_step's tuning stamps: none)
};

// member `member` of the team training universe U (U.team_w members)
template <int G, int VEC, int KCH, int NT>
__device__ __forceinline__ void universe_run_team(const UniverseDev &U, int member, int p_norm, int norm_flag, int opt,
                                                  int neg, int bern, int filter, const UniverseLaunch &cfg,
                                                  const UniShared &S) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = NT / G;
    constexpr bool PF = G >= 32;
    constexpr bool kFastUpd = uni_fast(G, VEC * KCH);
    const int W = (int)U.team_w;
    const int tid = threadIdx.x, lane = tid % G, grp = tid / G;
    const int bs = (int)U.bs, threads = (int)U.threads, D = (int)U.dim;
    const int E = (int)U.g.ent_total, R = (int)U.g.rel_total;
    const int seq = bs * (1 + neg), per_pos = neg + 2, nslots = bs * per_pos;
    const int nbatches = (int)U.nbatches, epochs = (int)U.epochs;
    const int pchunk = (int)(cfg.pchunk < U.nbatches ? cfg.pchunk : U.nbatches);
    int &s_count = *S.count;
    int &s_mcount = *S.ccount;
    float &s_loss = *S.loss;
    uint64_t *s_states = S.states;
    // LDS: list[list_cap] | mine[list_cap] | rflag[R] | head[E] | next[nslots] | batches [3][pchunk][seq] | grel [R][D]
    auto a4 = [](int v) { return (v + 3) & ~3; };
    int32_t *p = S.dyn;
    int32_t *s_list = p;
    p += a4((int)cfg.list_cap);
    int32_t *s_mine = p;
    p += a4((int)cfg.list_cap);
    int32_t *s_rflag = p;
    p += a4(R);
    int32_t *s_head = p;
    p += a4(E);
    int32_t *s_next = p;
    p += a4(nslots);
    int32_t *s_bh = p, *s_br = p + pchunk * seq, *s_bt = p + 2 * pchunk * seq;
    p += 3 * pchunk * seq;
    float *s_grel = reinterpret_cast<float *>(p);

    if (tid < threads) s_states[tid] = U.states[tid];
    const int per = bs % threads == 0 ? bs / threads : bs / threads + 1;
    const int rem = per > 0 ? bs - (bs / per) * per : 0;
    const int dpp = 1 + 2 * neg;
    const bool fastpre = per <= kPreJ && pchunk <= kPreC;
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
    for (int i = tid; i < R; i += NT) s_rflag[i] = 0;
    for (int i = tid; i < E; i += NT) s_head[i] = -1;
    for (int i = tid; i < R * D; i += NT) s_grel[i] = 0.f;
    StepParams P{};
    P.model = 0; P.p_norm = p_norm; P.norm_flag = norm_flag; P.opt = opt;
    P.lr = U.lr; P.margin = U.margin;
    P.ent_total = E; P.rel_total = R; P.dim = D;
    P.ent = U.ent; P.rel = U.rel; P.normv = nullptr;
    P.batch_size = bs; P.neg = neg;
    P.inv_count = 1.0f / (float)(bs * neg);
    const __amdgpu_buffer_rsrc_t r_ent = make_rsrc(U.ent, (uint32_t)(E * D * 4));
    const __amdgpu_buffer_rsrc_t r_rel = make_rsrc(U.rel, (uint32_t)(R * D * 4));
    const __amdgpu_buffer_rsrc_t r_eacc = make_rsrc(U.ent_acc, (uint32_t)(E * D * 4));
    const __amdgpu_buffer_rsrc_t r_racc = make_rsrc(U.rel_acc, (uint32_t)(R * D * 4));
    const __amdgpu_buffer_rsrc_t r_con = make_rsrc(U.contrib, (uint32_t)(nslots * D * 4));
    // team_part: [W][R][D] relation partials, then [W][epochs] loss partials
    const __amdgpu_buffer_rsrc_t r_part = make_rsrc(U.team_part, (uint32_t)(W * R * D * 4));
    float *loss_part = U.team_part + (int64_t)W * R * D;
    const TeamSink sink0{r_con, s_grel};
    const DeviceGraph &g = U.g;
    const Presampler<NT> presample{g, s_states, S.pre, fm_n, fm_e, threads, bs, neg, bern, filter, dpp, per, seq,
                                   fastpre, s_bh, s_br, s_bt};
    uint32_t arrivals = 0;
    float epoch_loss = 0.f;
    uint64_t t_pre = 0, t_a = 0, t_b = 0, t0 = 0, rows_b = 0;
    const bool prof = U.prof && member == 0;
    const uint64_t w_start = prof ? wall_clock64() : 0;
    __syncthreads();
    for (int epoch = 0; epoch < epochs; ++epoch) {
        for (int step = 0; step < nbatches; ++step) {
            if (prof) t0 = clock64();
            const int cs = step % pchunk;
            if (cs == 0) presample.draw(nbatches - step < pchunk ? nbatches - step : pchunk);
            if (tid == 0) {
                s_count = 0;
                s_mcount = 0;
                s_loss = 0.f;
            }
            __syncthreads();
            const int32_t *bh = s_bh + cs * seq, *br = s_br + cs * seq, *bt = s_bt + cs * seq;
            // link pass: the step's entity rows -> their static slots, the step's rows, this member's rows
            for (int q = tid; q < nslots; q += NT) {
                const int b = q / per_pos, k = q - b * per_pos;
                const int hp = bh[b];
                int row;
                if (k < neg) {
                    const int o = (k + 1) * bs + b;
                    row = bh[o] == hp ? bt[o] : bh[o];   // a negative shares one side with its positive
                } else {
                    row = k == neg ? hp : bt[b];
                }
                const int32_t prev = atomicExch(s_head + row, q);
                s_next[q] = prev;
                if (prev < 0) {
                    s_list[atomicAdd(&s_count, 1)] = row << 2;
                    if (row % W == member) s_mine[atomicAdd(&s_mcount, 1)] = row << 2;
                }
            }
            for (int b = tid; b < bs; b += NT) {
                const int r = br[b];
                if (atomicExch(s_rflag + r, 1) == 0) {
                    s_list[atomicAdd(&s_count, 1)] = (r << 2) | 1;
                    if (r % W == member) s_mine[atomicAdd(&s_mcount, 1)] = (r << 2) | 1;
                }
            }
            __syncthreads();
            if (prof) {
                const uint64_t t1 = clock64();
                t_pre += t1 - t0;
                t0 = t1;
            }
            // ---- phase A: this member's positives
            float lacc = 0.f;
            for (int j = grp; j * W + member < bs; j += GPB) {
                const int b = j * W + member;
                const int hq[1] = {bh[b]}, rq[1] = {br[b]}, tq[1] = {bt[b]};
                TeamSink sk0 = sink0;
                sk0.slot = b * per_pos;
                const TeamSink sk[1] = {sk0};
                const int hp = hq[0];
                lacc += transe_step<1, G, VEC, KCH, PF, true, true>(
                    P, hq, rq, tq, neg,
                    [&](int, int k, int &e, bool &tail_side) {
                        const int o = (k + 1) * bs + b;
                        tail_side = bh[o] == hp;
                        e = tail_side ? bt[o] : bh[o];
                    },
                    sk, lane);
            }
            if (lane == 0 && grp * W + member < bs) atomicAdd(&s_loss, lacc);
            __syncthreads();
            // this member's partial of every relation row of the step (zero where its positives did not touch it)
            const int n = s_count;
            for (int i = grp; i < n; i += GPB) {
                const int32_t code = s_list[i];
                if ((code & 3) != 1) continue;
                const int r = code >> 2;
                Vec gr;
                vload(gr, (const lfloat *)(s_grel + r * D), D, lane);
                bstore<G, VEC, KCH, 16>(gr, r_part, (uint32_t)((member * R + r) * D * 4), D, lane);
                Vec z;
                vzero(z);
                vstore(z, (lfloat *)(s_grel + r * D), D, lane);
            }
            arrivals += (uint32_t)W;
            team_barrier(U.team_sync, arrivals, U.team_err);
            if (prof) {
                const uint64_t t1 = clock64();
                t_a += t1 - t0;
                t0 = t1;
            }
            // ---- phase B: the rows this member owns
            const int nm = s_mcount;
            if (prof) rows_b += (uint64_t)nm;
            for (int i = grp; i < nm; i += GPB) {
                const int32_t code = s_mine[i];
                const int table = code & 3, row = code >> 2;
                const __amdgpu_buffer_rsrc_t rw = table == 0 ? r_ent : r_rel, ra = table == 0 ? r_eacc : r_racc;
                const uint32_t off = (uint32_t)(row * D * 4);
                Vec x, a, gs, y;
                bload<G, VEC, KCH, 16>(x, rw, off, D, lane);
                if (opt != 0) bload<G, VEC, KCH, 16>(a, ra, off, D, lane);
                if (table == 0) {
                    // the row's slots along its list, the first two loaded with the row
                    const int32_t c0 = s_head[row];
                    bload<G, VEC, KCH, 16>(gs, r_con, (uint32_t)(c0 * D * 4), D, lane);
                    int32_t c = s_next[c0];
                    if (c >= 0) {
                        bload<G, VEC, KCH, 16>(y, r_con, (uint32_t)(c * D * 4), D, lane);
#pragma unroll
                        for (int j = 0; j < Vec::N; ++j) gs.x[j] += y.x[j];
                        for (c = s_next[c]; c >= 0; c = s_next[c]) {
                            bload<G, VEC, KCH, 16>(y, r_con, (uint32_t)(c * D * 4), D, lane);
#pragma unroll
                            for (int j = 0; j < Vec::N; ++j) gs.x[j] += y.x[j];
                        }
                    }
                } else {
                    // the members' partials, in member order
                    bload<G, VEC, KCH, 16>(gs, r_part, (uint32_t)(row * D * 4), D, lane);
                    for (int m = 1; m < W; ++m) {
                        bload<G, VEC, KCH, 16>(y, r_part, (uint32_t)((m * R + row) * D * 4), D, lane);
#pragma unroll
                        for (int j = 0; j < Vec::N; ++j) gs.x[j] += y.x[j];
                    }
                }
                // TransE: entity and relation rows carry normalized-space gradients
                Vec gg;
                if (norm_flag) {
                    const float nx = fsqrt<kFastUpd>(vdot(x, x));
                    unormalize_bwd<kFastUpd>(x, nx, gs, gg);
                } else {
                    gg = gs;
                }
                if (opt == 0) {
#pragma unroll
                    for (int j = 0; j < Vec::N; ++j) x.x[j] = x.x[j] + (-U.lr) * gg.x[j];
                } else {
#pragma unroll
                    for (int j = 0; j < Vec::N; ++j) {
                        a.x[j] = a.x[j] + gg.x[j] * gg.x[j];
                        if constexpr (kFastUpd)
                            x.x[j] = x.x[j] + (-U.lr) * (gg.x[j] * frcp<true>(fsqrt<true>(a.x[j]) + 1e-10f));
                        else
                            x.x[j] = x.x[j] + (-U.lr) * gg.x[j] / (sqrtf(a.x[j]) + 1e-10f);
                    }
                    bstore<G, VEC, KCH, 16>(a, ra, off, D, lane);
                }
                bstore<G, VEC, KCH, 16>(x, rw, off, D, lane);
            }
            __syncthreads();   // (the heads are read above by other lane groups)
            for (int i = tid; i < n; i += NT) {
                const int32_t code = s_list[i];
                if ((code & 3) == 0) s_head[code >> 2] = -1; else s_rflag[code >> 2] = 0;
            }
            if (tid == 0) epoch_loss += s_loss * P.inv_count + (member == 0 ? U.margin : 0.f);
            arrivals += (uint32_t)W;
            team_barrier(U.team_sync, arrivals, U.team_err);
            if (prof) {
                const uint64_t t1 = clock64();
                t_b += t1 - t0;
            }
        }
        if (tid == 0) {   // this member's part of the epoch's loss sum
            __hip_atomic_store(loss_part + member * epochs + epoch, epoch_loss, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        epoch_loss = 0.f;
    }
    arrivals += (uint32_t)W;
    team_barrier(U.team_sync, arrivals, U.team_err);
    if (member == 0) {
        if (tid < epochs && U.losses) {
            float l = 0.f;
            for (int m = 0; m < W; ++m)
                l += __hip_atomic_load(loss_part + m * epochs + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            U.losses[tid] = l;
        }
        if (tid < threads) U.states[tid] = s_states[tid];
        if (prof && tid == 0) {
            U.prof[0] = t_pre;
            U.prof[1] = t_a;
            U.prof[2] = t_b;
            U.prof[3] = (uint64_t)U.epochs * U.nbatches;
            U.prof[4] = (uint64_t)bs;
            U.prof[5] = (uint64_t)D;
            U.prof[6] = (uint64_t)E;
            U.prof[7] = (w_start << 32) | ((wall_clock64() - w_start) & 0xffffffffull);
            U.prof[62] = rows_b;   // (member 0's rows)
        }
    }
}

// One launch of team universes of one row shape: workgroup b is member map[2b + 1] of universe map[2b] (-1: idle)
template <int NT, int SHAPE, int G, int VEC, int KCH>
__global__ __launch_bounds__(NT, NT / 512 * 2) void k_universes_team(const UniverseDev *__restrict__ us,
                                                                       const int32_t *__restrict__ map, int p_norm,
                                                                       int norm_flag, int opt, int64_t neg, int bern,
                                                                       int filter, UniverseLaunch cfg) {
    extern __shared__ int32_t s_dyn[];
    __shared__ uint64_t s_states[64];
    __shared__ int s_count, s_ccount;
    __shared__ float s_loss;
    __shared__ PreTables s_pre;
    const int u = __builtin_amdgcn_readfirstlane(map[2 * blockIdx.x]);
    const int member = __builtin_amdgcn_readfirstlane(map[2 * blockIdx.x + 1]);
    if (member < 0) return;
    const UniShared S{s_dyn, s_states, &s_count, &s_ccount, &s_loss, &s_pre};
    const UniverseDev U = us[u];
    universe_run_team<G, VEC, KCH, NT>(U, member, p_norm, norm_flag, opt, (int)neg, bern, filter, cfg, S);
}

}  // namespace dev
}  // namespace pt
