// Team universes: one universe trained by a TEAM of W workgroups on W CUs (TransE, the 1,024-thread row shapes).
//
// A universe's training is a chain of ~epochs x 20 dependent minibatch steps (Parallel_Universe_Config.py:228-258),
// and one workgroup runs it (universes_kern.h). When a GPU holds fewer universes than CUs - the BASELINE PU configs
// at 8 GPUs: C4 128, C3 64, C5 32 universes per GPU on 256 CUs - the set's makespan is its longest chain and most
// CUs idle. A team splits each step of one universe over its members:
//
//   presample  every member draws the same batches into its own LDS (presample_draw, as universe_run: no exchange);
//   link pass  every member links the step's entity rows to their STATIC contribution slots (slot b * (neg + 2) + k:
//              negative k, then the head and tail rows of positive b) in its own LDS lists and maps the step's
//              relations to LDS gradient rows, from the batch alone; it collects the step's rows - the same sets on
//              every member, each member also the rows it owns (entity / relation id mod W);
//   phase A    member m runs positives b = m, m + W, ... (transe_step with ALWAYS: every slot of a positive is
//              written, zero rows for an inactive pair), relation gradients into its LDS rows, which it publishes as
//              its partials of the step's relations;
//   barrier    (team_barrier)
//   phase B    member m updates the rows it owns: an entity row the sum of its slots along its list (list_sum, four
//              rows in flight), a relation row the W members' partials; normalize Jacobian of the pre-step row,
//              Adagrad / SGD;
//   barrier.
// Every exchanged byte (contribution rows, relation partials, the universe's table rows and Adagrad state, loss
// partials) is stored, drained (vmcnt(0)) before the arrival atomic, and read with sc1 buffer loads (past the CU's L1,
// served by the XCD's L2). Where the members run decides the store form: the host places a team's members on blocks of
// one residue mod 8 (the dispatcher's round-robin over the XCDs) and each member reads its XCD (HW_REG_XCC_ID) at the
// start; when all members share one XCD - one L2 - the stores are plain (the lines stay in that L2), otherwise sc1
// write-through stores, the hand-off form of MI355X_MICROARCH.md ("Inter-workgroup visibility") that holds wherever the
// members run. (sc1 stores drop the line from the L2: every later read of a table row then crosses the fabric - the
// all-sc1 form measured 2x slower per step, round 6.)
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

// a row store of a team member: plain when the team shares one L2 (coh), else sc1 write-through
template <int G, int VEC, int KCH>
__device__ __forceinline__ void tstore(bool coh, const V<G, VEC, KCH> &o, __amdgpu_buffer_rsrc_t rs, uint32_t off, int D,
                                       int lane) {
    if (coh)
        bstore<G, VEC, KCH, 0>(o, rs, off, D, lane);
    else
        bstore<G, VEC, KCH, 16>(o, rs, off, D, lane);
}

// gradient sink of a team member: entity rows to the positive's next static slot, relation rows into the member's LDS
// rows of the step's relations (its partials: published after phase A)
struct TeamSink {
    __amdgpu_buffer_rsrc_t contrib;
    bool coh;                    // the team shares one XCD
    float *grel;                 // LDS [rel_step][D]
    const int32_t *rmap;         // LDS [R]: relation -> its row among the step's relations
    mutable int slot = 0;
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void ent(int, const V<G, VEC, KCH> &g, int D, int lane) const {
        tstore(coh, g, contrib, (uint32_t)(slot++ * D * 4), D, lane);
    }
    template <int G, int VEC, int KCH>
    __device__ __forceinline__ void rel(int row, const V<G, VEC, KCH> &g, int D, int lane) const {
        vatomic(g, (lfloat *)(grel + ((const lint32 *)rmap)[row] * D), D, lane);
    }
    uint64_t *trace = nullptr;   // (transe_step's tuning stamps: none)
};

// member `member` of the team training universe U (T.w members). A positive b owns the static entity slots
// b * (neg + 2) + k: its negatives k < neg, then its head and tail rows (transe_step's sink order).
template <int G, int VEC, int KCH, int NT>
__device__ __forceinline__ void universe_run_team(const UniverseDev &U, const TeamDev &T, int member, int p_norm,
                                                  int norm_flag, int opt, int neg, int bern, int filter,
                                                  const UniverseLaunch &cfg, const UniShared &S) {
    using Vec = V<G, VEC, KCH>;
    constexpr int GPB = NT / G;
    constexpr bool PF = G >= 32;
    constexpr bool kFastUpd = uni_fast(G, VEC * KCH);
    const int W = (int)T.w;
    const int tid = threadIdx.x, lane = tid % G, grp = tid / G;
    const int bs = (int)U.bs, threads = (int)U.threads, D = (int)U.dim;
    const int E = (int)U.g.ent_total, R = (int)U.g.rel_total;
    const int seq = bs * (1 + neg), per_pos = neg + 2, nslots = bs * per_pos;
    const int rstep = R < bs ? R : bs;   // the step's relations, at most
    const int nbatches = (int)U.nbatches, epochs = (int)U.epochs;
    const int pchunk = (int)(cfg.pchunk < U.nbatches ? cfg.pchunk : U.nbatches);
    int &s_count = *S.count;
    int &s_mcount = *S.ccount;
    float &s_loss = *S.loss;
    uint64_t *s_states = S.states;
    // LDS: list[cap] | mine[cap] | head[E] | rmap[R] | rlist[rstep] | next[nslots] | batches [3][pchunk][seq] |
    //      grel [rstep][D]
    auto a4 = [](int v) { return (v + 3) & ~3; };
    int32_t *p = S.dyn;
    int32_t *s_list = p;
    p += a4((int)cfg.list_cap);
    int32_t *s_mine = p;
    p += a4((int)cfg.list_cap);
    int32_t *s_head = p;
    p += a4(E);
    int32_t *s_rmap = p;
    p += a4(R);
    int32_t *s_rlist = p;
    p += a4(rstep);
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
        PreTables &PT = *S.pre;
        if (tid < kPreJ) {
            PT.j[tid] = lcg_power((uint64_t)tid * (uint64_t)dpp);
        } else if (tid < kPreJ + 2 * kPreC) {
            const int c = (tid - kPreJ) >> 1, w = (tid - kPreJ) & 1;
            PT.c[c][w] = lcg_power((uint64_t)c * (uint64_t)(w ? rem : per) * (uint64_t)dpp);
        }
    }
    const FastMod fm_n = fastmod_make((uint64_t)U.g.train_total), fm_e = fastmod_make((uint64_t)(E - 1));
    for (int i = tid; i < E; i += NT) s_head[i] = -1;
    for (int i = tid; i < R; i += NT) s_rmap[i] = -1;
    for (int i = tid; i < rstep * D; i += NT) s_grel[i] = 0.f;
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
    const __amdgpu_buffer_rsrc_t r_part = make_rsrc(T.part, (uint32_t)(W * R * D * 4));
    float *loss_part = T.part + W * R * D;
    uint32_t *xcc_tab = reinterpret_cast<uint32_t *>(loss_part + W * epochs);
    uint32_t arrivals = 0;
    // the members' XCDs: plain stores when the whole team shares one L2 (see the file comment)
    if (tid == 0)
        __hip_atomic_store(xcc_tab + member, (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    arrivals += (uint32_t)W;
    team_barrier(T.sync, arrivals, T.err);
    bool coh = true;
    {
        const uint32_t x0 = __hip_atomic_load(xcc_tab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int m = 1; m < W; ++m)
            coh = coh && __hip_atomic_load(xcc_tab + m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == x0;
    }
    coh = __builtin_amdgcn_readfirstlane((int)coh) != 0;
    const TeamSink sink0{r_con, coh, s_grel, s_rmap};
    const DeviceGraph &g = U.g;
    float epoch_loss = 0.f;
    uint64_t t_pre = 0, t_a = 0, t_b = 0, t0 = 0, rows_b = 0, t_bar = 0;
    const bool prof = U.prof && member == 0;
    const uint64_t w_start = prof ? wall_clock64() : 0;
    __syncthreads();
    for (int epoch = 0; epoch < epochs; ++epoch) {
        for (int step = 0; step < nbatches; ++step) {
            if (prof) t0 = clock64();
            const int cs = step % pchunk;
            if (cs == 0)
                presample_draw<NT>(nbatches - step < pchunk ? nbatches - step : pchunk, g, s_states, S.pre, fm_n, fm_e,
                                   threads, bs, neg, bern, filter, dpp, per, seq, fastpre, s_bh, s_br, s_bt);
            if (tid == 0) {
                s_count = 0;
                s_mcount = 0;
                *S.rcount = 0;
                s_loss = 0.f;
            }
            __syncthreads();
            const int32_t *bh = s_bh + cs * seq, *br = s_br + cs * seq, *bt = s_bt + cs * seq;
            // link pass: the step's entity rows -> their static slots; the step's relations -> their LDS rows; the
            // step's rows and this member's rows (entity / relation id mod W)
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
                if (atomicCAS(s_rmap + r, -1, -2) == -1) {
                    const int ix = atomicAdd(S.rcount, 1);
                    s_rmap[r] = ix;
                    s_rlist[ix] = r;
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
            // this member's partial of each of the step's relation rows (zero where its positives did not touch it)
            const int nr = *S.rcount;
            for (int ix = grp; ix < nr; ix += GPB) {
                const int r = s_rlist[ix];
                Vec gr;
                vload(gr, (const lfloat *)(s_grel + ix * D), D, lane);
                tstore(coh, gr, r_part, (uint32_t)((member * R + r) * D * 4), D, lane);
                Vec z;
                vzero(z);
                vstore(z, (lfloat *)(s_grel + ix * D), D, lane);
            }
            arrivals += (uint32_t)W;
            const uint64_t tb0 = prof ? clock64() : 0;
            team_barrier(T.sync, arrivals, T.err);
            if (prof) {
                const uint64_t t1 = clock64();
                t_bar += t1 - tb0;
                t_a += t1 - t0;
                t0 = t1;
            }
            // ---- phase B: the rows this member owns - an entity row the sum of its slots along its list (four rows
            // in flight), a relation row the members' partials in member order
            const int n = s_count, nm = s_mcount;
            if (prof) rows_b += (uint64_t)nm;
            for (int i = grp; i < nm; i += GPB) {
                const int32_t code = s_mine[i];
                const int table = code & 3, row = code >> 2;
                const __amdgpu_buffer_rsrc_t rw = table == 0 ? r_ent : r_rel, ra = table == 0 ? r_eacc : r_racc;
                const uint32_t off = (uint32_t)(row * D * 4);
                Vec x, a, gs;
                bload<G, VEC, KCH, 16>(x, rw, off, D, lane);
                if (opt != 0) bload<G, VEC, KCH, 16>(a, ra, off, D, lane);
                if (table == 0) {
                    vzero(gs);
                    list_sum<4>(gs, s_head[row], s_next, [&](Vec &rr, int32_t c) {
                        bload<G, VEC, KCH, 16>(rr, r_con, (uint32_t)(c * D * 4), D, lane);
                    });
                } else {
                    Vec y[4];
                    bload<G, VEC, KCH, 16>(gs, r_part, (uint32_t)(row * D * 4), D, lane);
#pragma unroll
                    for (int m = 1; m < 4; ++m)
                        if (m < W) bload<G, VEC, KCH, 16>(y[m], r_part, (uint32_t)((m * R + row) * D * 4), D, lane);
#pragma unroll
                    for (int m = 1; m < 4; ++m)
                        if (m < W) {
#pragma unroll
                            for (int j = 0; j < Vec::N; ++j) gs.x[j] += y[m].x[j];
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
                    tstore(coh, a, ra, off, D, lane);
                }
                tstore(coh, x, rw, off, D, lane);
            }
            __syncthreads();   // (the heads are read above by other lane groups)
            for (int i = tid; i < n; i += NT) {
                const int32_t code = s_list[i];
                if ((code & 3) == 0) s_head[code >> 2] = -1; else s_rmap[code >> 2] = -1;
            }
            if (tid == 0) epoch_loss += s_loss * P.inv_count + (member == 0 ? U.margin : 0.f);
            arrivals += (uint32_t)W;
            const uint64_t tb1 = prof ? clock64() : 0;
            team_barrier(T.sync, arrivals, T.err);
            if (prof) {
                const uint64_t t1 = clock64();
                t_bar += t1 - tb1;
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
    team_barrier(T.sync, arrivals, T.err);
    if (member == 0) {
        for (int e = tid; U.losses && e < epochs; e += NT) {
            float l = 0.f;
            for (int m = 0; m < W; ++m)
                l += __hip_atomic_load(loss_part + m * epochs + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            U.losses[e] = l;
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
            U.prof[60] = ((uint64_t)W << 32) | (coh ? 1u : 0u);   // team width, one XCD
            U.prof[61] = t_bar;    // cycles member 0 spent in the two team barriers of its steps
            U.prof[62] = rows_b;   // (member 0's rows)
        }
    }
}

// One launch of team universes of one row shape: workgroup b is member map[2b + 1] of universe map[2b] (-1: idle)
template <int NT, int SHAPE, int G, int VEC, int KCH>
__global__ __launch_bounds__(NT, NT / 512 * 2) void k_universes_team(const UniverseDev *__restrict__ us,
                                                                       const TeamDev *__restrict__ teams,
                                                                       const int32_t *__restrict__ map, int p_norm,
                                                                       int norm_flag, int opt, int64_t neg, int bern,
                                                                       int filter, UniverseLaunch cfg) {
    extern __shared__ int32_t s_dyn[];
    __shared__ uint64_t s_states[64];
    __shared__ int s_count, s_ccount, s_rcount;
    __shared__ float s_loss;
    __shared__ PreTables s_pre;
    const int u = __builtin_amdgcn_readfirstlane(map[2 * blockIdx.x]);
    const int member = __builtin_amdgcn_readfirstlane(map[2 * blockIdx.x + 1]);
    if (member < 0) return;
    const UniShared S{s_dyn, s_states, &s_count, &s_ccount, &s_loss, &s_pre, &s_rcount};
    const UniverseDev U = us[u];
    const TeamDev T = teams[u];
    universe_run_team<G, VEC, KCH, NT>(U, T, member, p_norm, norm_flag, opt, (int)neg, bern, filter, cfg, S);
}

}  // namespace dev
}  // namespace pt
