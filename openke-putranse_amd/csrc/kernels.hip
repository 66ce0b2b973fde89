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

#include "tuning.h"
#include "device.h"
#include "graph.h"
#include "kernels.h"
#include "rng.h"

namespace pt {
namespace dev {
using pt::CsrWork;


// sampling() into arrays (one thread per positive, Base.cpp:185-264); the stream advance is a separate
// kernel. mode 0: a coin per negative picks the replaced side (draw_negative); mode -1 (sampling_head)
// replaces the head via corrupt_tail, mode 1 (sampling_tail) the tail via corrupt_head - no coin, and
// corrupt_*'s default filter_flag = true (Base.cpp:233-245). Then neg_rel relation corruptions
// (corrupt_rel, p = false, filter_flag = true: Corrupt.h:108-135, :179-189) drawn among the relations
// not yet linking (h, t) - the same run search as the entity corruptions, over the cmp_rel list.
__global__ void k_sample(DeviceGraph g, const uint64_t *__restrict__ states, int64_t threads, int64_t bs, int64_t neg,
                         int64_t neg_rel, int mode, int bern, int filter, int64_t *__restrict__ oh,
                         int64_t *__restrict__ ot, int64_t *__restrict__ orr, float *__restrict__ oy) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= bs) return;
    const int64_t per_neg = mode == 0 ? 2 : 1;
    const PosDraw pd = draw_positive(g, states, threads, bs, b, 1 + per_neg * neg + neg_rel);
    const int64_t hp = pd.h, rp = pd.r, tp = pd.t;
    oh[b] = hp; ot[b] = tp; orr[b] = rp;
    if (oy) oy[b] = 1.f;
    for (int64_t k = 0; k < neg; ++k) {
        int64_t hh = hp, tt = tp;
        if (mode == 0) {
            int tail_side;
            const int64_t e = draw_negative(g, pd, k, bern, filter, &tail_side);
            if (tail_side) tt = e; else hh = e;
        } else {
            uint64_t s = lcg_jump(pd.s1, (uint64_t)k);
            if (mode < 0) hh = corrupt_in_run(g.tail_h, pd.tr_lo, pd.tr_hi, g.ent_total, s);
            else tt = corrupt_in_run(g.head_t, pd.hr_lo, pd.hr_hi, g.ent_total, s);
        }
        const int64_t o = (k + 1) * bs + b;
        oh[o] = hh;
        ot[o] = tt;
        orr[o] = rp;
        if (oy) oy[o] = -1.f;
    }
    if (neg_rel > 0) {
        const int2 run = g.ht_run[pd.idx];
        for (int64_t k = 0; k < neg_rel; ++k) {
            uint64_t s = lcg_jump(pd.s1, (uint64_t)(per_neg * neg + k));
            const int64_t o = (neg + k + 1) * bs + b;
            oh[o] = hp;
            ot[o] = tp;
            orr[o] = corrupt_in_run(g.rel_r, run.x, run.y, g.rel_total, s);
            if (oy) oy[o] = -1.f;
        }
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

// the fused step + apply's row-use counts (CsrWork::uses): the positive's h and t rows and its relation row
__device__ __forceinline__ void count_uses(const CsrWork &w, int64_t call, const PosDraw &pd) {
    if (!w.uses) return;
    int32_t *u = w.uses + call * w.use_stride;
    atomicAdd(u + pd.h, 1);
    atomicAdd(u + pd.t, 1);
    atomicAdd(u + w.rel_base + pd.r, 1);
}

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
        count_uses(w, call, pd);
        return;
    }
    int side;
    const int64_t e = draw_negative(g, pd, k, bern, filter, &side);
    const int64_t o = call * bs * neg + b * neg + k;
    w.neg[o] = (int32_t)((e << 1) | side);
    w.off[o] = atomicAdd(&w.cnt[call * w.cnt_stride + e], 1);
}

// The split sampler's cross-workgroup exchange (k_sample_part): relaxed read-modify-writes at AGENT scope,
// spelled out. Agent-scope atomics are performed at the device's coherence point (not in an XCD's L2), so
// every part's count adds and ticket are seen by the last part whatever XCDs the parts run on; nothing else
// the parts share inside the launch is read before a kernel boundary.
__device__ __forceinline__ int32_t agent_add(int32_t *p, int32_t v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t agent_exch(int32_t *p, int32_t v) {
    return __hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One negative slot's draw from its positive's LDS record (k_sample_sort, k_sample_part): the coin and the
// corruption draw of draw_negative with the same stream offsets and arithmetic; when the drawn index
// falls inside the known-entity run, the boundary search over it (corrupt_in_run) is left to the caller
// (q open; otherwise q is closed and e is the entity).
struct SlotDraw {
    RunSearch q;
    int64_t e;
    int side;
    bool search;
};

// jump maps of the LCG by 2k draws for k < kJumpTab, staged in LDS once per workgroup: a slot's stream
// start is then one 64-bit multiply-add away from its positive's state instead of a square-and-multiply
// loop (the loop remains for k >= kJumpTab)
constexpr int kJumpTab = 256;
__device__ __forceinline__ int32_t jump_tab_len(int64_t neg) { return neg < kJumpTab ? (int32_t)neg : kJumpTab; }
template <int NT>
__device__ __forceinline__ void jump_tab_fill(Affine *jt, int64_t neg, int tid) {
    for (int32_t k = tid; k < jump_tab_len(neg); k += NT) jt[k] = lcg_power((uint64_t)(2 * k));
}

__device__ __forceinline__ SlotDraw slot_prepare(const int32_t *q, int32_t k, int64_t E, int filter,
                                                 const DeviceGraph &g, const Affine *jt, int dbg = 0) {
    SlotDraw d;
    const uint64_t s1 = *reinterpret_cast<const uint64_t *>(q + 10);
    uint64_t s;
    if (PT_ABLATE(dbg, 2)) s = s1 + k;
    else if (k < kJumpTab) { const Affine m = jt[k]; s = m.a * s1 + m.c; }
    else s = lcg_jump(s1, (uint64_t)(2 * k));
    d.side = (float)(lcg_next(s) % 1000ULL) < __int_as_float(q[0]) ? 1 : 0;
    d.search = false;
    d.q.l = 0;
    d.q.r = 1;   // closed
    if (filter) {
        const int32_t *vals = d.side ? g.head_t : g.tail_h;
        const int32_t lo = d.side ? q[1] : q[3], hi = d.side ? q[2] : q[4];
        const int32_t vlo = d.side ? q[5] : q[7], vhi = d.side ? q[6] : q[8];
        const int64_t tmp = PT_ABLATE(dbg, 4) ? (int64_t)((uint32_t)lcg_next(s) & 8191) : rand_max(s, E - (hi - lo + 1));
        if (tmp < vlo) d.e = tmp;
        else if (tmp > vhi - hi + lo - 1) d.e = tmp + hi - lo + 1;
        else if (PT_ABLATE(dbg, 1)) d.e = tmp;
        else { d.search = true; d.q = run_search(vals, lo, hi, vlo, vhi, (int32_t)tmp); d.e = 0; }
    } else {
        const int64_t tmp = rand_max(s, E - 1);
        const int64_t skip = d.side ? q[5] : q[6];
        d.e = tmp < skip ? tmp : tmp + 1;
    }
    return d;
}

// two slots' boundary searches stepped in lock step (both gathers in flight together)
__device__ __forceinline__ void slot_search2(SlotDraw &d0, SlotDraw &d1) {
    for (;;) {
        const bool a0 = rs_open(d0.q), a1 = rs_open(d1.q);
        if (!(a0 || a1)) break;
        const int32_t m0 = a0 ? rs_probe(d0.q) : 0, m1 = a1 ? rs_probe(d1.q) : 0;
        const int32_t v0 = a0 ? d0.q.vals[m0] : 0, v1 = a1 ? d1.q.vals[m1] : 0;   // only open searches load
        if (a0) rs_update(d0.q, m0, v0);
        if (a1) rs_update(d1.q, m1, v1);
    }
    if (d0.search) d0.e = rs_entity(d0.q);
    if (d1.search) d1.e = rs_entity(d1.q);
}

// SL slots' boundary searches in lock step
template <int SL>
__device__ __forceinline__ void slot_searchN(SlotDraw (&d)[SL]) {
    for (;;) {
        bool a[SL], any = false;
#pragma unroll
        for (int i = 0; i < SL; ++i) { a[i] = rs_open(d[i].q); any |= a[i]; }
        if (!any) break;
        int32_t m[SL], v[SL];
#pragma unroll
        for (int i = 0; i < SL; ++i) m[i] = a[i] ? rs_probe(d[i].q) : 0;
#pragma unroll
        for (int i = 0; i < SL; ++i) v[i] = a[i] ? d[i].q.vals[m[i]] : 0;   // only open searches load
#pragma unroll
        for (int i = 0; i < SL; ++i)
            if (a[i]) rs_update(d[i].q, m[i], v[i]);
    }
#pragma unroll
    for (int i = 0; i < SL; ++i)
        if (d[i].search) d[i].e = rs_entity(d[i].q);
}

// Sampling + counting sort of one sampled call per workgroup, entirely in LDS (when the bucket counts
// and the call's positives fit): the positives are drawn once (not once per slot), every slot's
// negative reserves its rank with an LDS atomic, the counts are scanned in LDS and every slot's
// destination resolved - the same pos / neg / start / destination arrays as k_sample_csr +
// k_scan_counts, without the 52,000 returning global atomics per call and the second pass.
// The sampler streams are read only; the caller advances them afterwards (k_advance).
__global__ __launch_bounds__(1024) void k_sample_sort(DeviceGraph g, const uint64_t *__restrict__ states,
                                                      int64_t threads, int64_t bs, int64_t neg, int bern, int filter,
                                                      int64_t n, CsrWork w) {
    extern __shared__ __attribute__((aligned(16))) int32_t lds[];
    __shared__ int32_t wtot[16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t call = blockIdx.x;
    Affine *jt = reinterpret_cast<Affine *>(lds);                        // [jump_tab_len(neg)] jump maps
    int32_t *cnt = lds + 4 * jump_tab_len(neg);                          // [n] counts, then starts
    // per positive [12] int32: prob bits, hr_lo hr_hi tr_lo tr_hi, then (filter) the run bounds'
    // values head_t[hr_lo] head_t[hr_hi] tail_h[tr_lo] tail_h[tr_hi] or (no filter) h t, pad, stream state
    // after the index draw (8 B): every slot's draw needs global memory only inside a run's boundary search
    int32_t *pi = cnt + ((n + 3) & ~int64_t(3));
    for (int64_t i = tid; i < n; i += 1024) cnt[i] = 0;
    jump_tab_fill<1024>(jt, neg, tid);
    const int64_t dpp = 1 + 2 * neg;
    for (int64_t b = tid; b < bs; b += 1024) {
        const PosDraw pd = draw_positive(g, states, threads, bs, b, dpp, call);
        int32_t *q = pi + 12 * b;
        q[0] = __float_as_int(bern ? g.bern_prob[pd.r] : 500.f);
        q[1] = pd.hr_lo; q[2] = pd.hr_hi; q[3] = pd.tr_lo; q[4] = pd.tr_hi;
        if (filter) {
            q[5] = g.head_t[pd.hr_lo]; q[6] = g.head_t[pd.hr_hi];
            q[7] = g.tail_h[pd.tr_lo]; q[8] = g.tail_h[pd.tr_hi];
        } else {
            q[5] = (int32_t)pd.h; q[6] = (int32_t)pd.t; q[7] = 0; q[8] = 0;
        }
        *reinterpret_cast<uint64_t *>(q + 10) = pd.s1;
        w.pos[call * bs + b] = make_int4((int)pd.h, (int)pd.r, (int)pd.t, 0);
        count_uses(w, call, pd);
    }
    __syncthreads();
    const int64_t slots = bs * neg;
    const int64_t E = g.ent_total;
    int32_t *nrec = w.neg + call * slots;
    int32_t *noff = w.off + call * slots;
    // slots o and o + 1024 per iteration (o = b * neg + k, walked with incremental (b, k) instead of a 64-bit
    // division per slot); their runs' boundary searches advance in lock step so both gathers are in
    // flight together. A missing second slot (past the end) draws and writes nothing.
    const int32_t neg32 = (int32_t)neg, db = 1024 / neg32, dk = 1024 - db * neg32;
    int32_t b = tid / neg32, k = tid - b * neg32;
    for (int64_t o = tid; o < slots; o += 2048) {
        int32_t b2 = b + db, k2 = k + dk;
        if (k2 >= neg32) { k2 -= neg32; ++b2; }
        const bool two = o + 1024 < slots;
        SlotDraw d0 = slot_prepare(pi + 12 * b, k, E, filter, g, jt);
        SlotDraw d1 = slot_prepare(pi + 12 * (two ? b2 : b), two ? k2 : k, E, filter, g, jt);
        if (!two) { d1.q.l = 0; d1.q.r = 1; d1.search = false; }   // no second slot: its search stays closed
        slot_search2(d0, d1);
        const int64_t e0 = d0.e;
        nrec[o] = (int32_t)((e0 << 1) | d0.side);
        noff[o] = atomicAdd(&cnt[e0], 1);
        if (two) {
            const int64_t e1 = d1.e;
            nrec[o + 1024] = (int32_t)((e1 << 1) | d1.side);
            noff[o + 1024] = atomicAdd(&cnt[e1], 1);
        }
        b = b2 + db; k = k2 + dk;
        if (k >= neg32) { k -= neg32; ++b; }
    }
    __syncthreads();
    // exclusive scan of cnt[0, n): contiguous chunks per thread, wave shuffles, LDS wave totals
    const int64_t per = (n + 1023) / 1024;
    const int64_t lo = tid * per, hi = lo + per < n ? lo + per : n;
    int32_t tsum = 0;
    for (int64_t i = lo; i < hi; ++i) tsum += cnt[i];
    int32_t incl = tsum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wtot[wid] = incl;
    __syncthreads();
    int32_t run = incl - tsum;
    for (int q = 0; q < wid; ++q) run += wtot[q];
    int32_t *start = w.start + call * w.start_stride;
    for (int64_t i = lo; i < hi; ++i) {
        const int32_t c = cnt[i];
        cnt[i] = run;
        start[i] = run;
        run += c;
    }
    if (tid == 1023) start[n] = run;   // the last thread's chunk ends at n (or is empty): run = total
    __syncthreads();
    for (int64_t o = tid; o < slots; o += 1024) noff[o] = cnt[nrec[o] >> 1] + noff[o];
}

// LDS bucket rank of entity e: 16-bit packed counts (two buckets per word; a part never holds 65536
// slots, so a half never carries into the other) or plain 32-bit counts
template <bool PACK>
__device__ __forceinline__ int32_t lds_rank(int32_t *cnt, int64_t e) {
    if constexpr (PACK) {
        const int sh = (int)(e & 1) << 4;
        return (atomicAdd(&cnt[e >> 1], 1 << sh) >> sh) & 0xffff;
    } else {
        return atomicAdd(&cnt[e], 1);
    }
}
template <bool PACK>
__device__ __forceinline__ int32_t lds_bucket(const int32_t *cnt, int64_t e) {
    if constexpr (PACK) return (cnt[e >> 1] >> ((int)(e & 1) << 4)) & 0xffff;
    else return cnt[e];
}

// Split sampling + counting sort: `parts` workgroups per sampled call (grid calls x parts), so a chunk
// of few steps still fills the chip (k_sample_sort runs one workgroup per call). Part p owns positives
// [p*bs/parts, (p+1)*bs/parts) of its call and all their slots. It draws them exactly as k_sample_sort
// does (positives once, per-positive constants in LDS, two slots per thread with lock-step run
// searches) and ranks every slot in an LDS count of its corrupted entity (16-bit packed counts when a
// call has < 65536 slots; the call's global counts are then packed the same way). It then reserves
// each touched bucket's range in the call's global counts with ONE returning atomic per touched count
// word and turns its slots' LDS ranks into ranks inside the call-wide buckets. The part whose ticket add comes last exchanges the global counts with zeros (atomics on
// both sides: every part's adds are seen, and the counts are clear for the next chunk) and scans them
// into start[]; the last call's last part then advances the sampler streams. off[] keeps the ranks
// (CsrWork::rank_only): the step kernel adds start[entity] when it loads a slot's record.
// A launch may sample calls [call0, call0 + gridDim.x / parts) of a chunk (`w` viewed at call0: its per-call
// arrays and tickets start there; the draws take their stream positions from call0 + call); advance = 0 leaves
// the stream advance to a later launch (k_advance), so two launches can sample one chunk side by side.
template <int NT, bool PACK, int SL>
__global__ __launch_bounds__(NT) void k_sample_part(DeviceGraph g, uint64_t *states,
                                                    int64_t threads, int64_t bs, int64_t neg, int bern, int filter,
                                                    int64_t parts, CsrWork w, int64_t call0, int advance) {
    extern __shared__ __attribute__((aligned(16))) int32_t lds[];
    __shared__ int32_t wtot[NT / 64];
    __shared__ int32_t is_last;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t call = blockIdx.x / parts, part = blockIdx.x - call * parts;
    const int64_t b0 = part * bs / parts, b1 = (part + 1) * bs / parts;
    const int64_t E = g.ent_total;
    const int64_t cwords = PACK ? (E + 1) >> 1 : E;
    uint64_t *prof = w.prof ? w.prof + 8 * (int64_t)blockIdx.x : nullptr;
#define PT_PHASE(i) if (prof && tid == 0) prof[i] = wall_clock64()
    PT_PHASE(0);
    Affine *jt = reinterpret_cast<Affine *>(lds);        // [jump_tab_len(neg)] jump maps
    int32_t *cnt = lds + 4 * jump_tab_len(neg);
    int32_t *pi = cnt + ((cwords + 3) & ~int64_t(3));    // [b1 - b0][12] positive records (k_sample_sort)
    for (int64_t i = tid; i < cwords; i += NT) cnt[i] = 0;
    jump_tab_fill<NT>(jt, neg, tid);
    const int64_t dpp = 1 + 2 * neg;
    for (int64_t b = b0 + tid; b < b1; b += NT) {
        const PosDraw pd = draw_positive(g, states, threads, bs, b, dpp, call0 + call);
        int32_t *q = pi + 12 * (b - b0);
        q[0] = __float_as_int(bern ? g.bern_prob[pd.r] : 500.f);
        q[1] = pd.hr_lo; q[2] = pd.hr_hi; q[3] = pd.tr_lo; q[4] = pd.tr_hi;
        if (filter) {
            q[5] = g.head_t[pd.hr_lo]; q[6] = g.head_t[pd.hr_hi];
            q[7] = g.tail_h[pd.tr_lo]; q[8] = g.tail_h[pd.tr_hi];
        } else {
            q[5] = (int32_t)pd.h; q[6] = (int32_t)pd.t; q[7] = 0; q[8] = 0;
        }
        *reinterpret_cast<uint64_t *>(q + 10) = pd.s1;
        w.pos[call * bs + b] = make_int4((int)pd.h, (int)pd.r, (int)pd.t, 0);
        count_uses(w, call, pd);
    }
    __syncthreads();
    PT_PHASE(1);
    const int64_t slots = bs * neg;
    int32_t *nrec = w.neg + call * slots;
    int32_t *noff = w.off + call * slots;
    const int64_t o0 = b0 * neg, o1 = b1 * neg;
    // thread tid takes slots o0 + tid + NT*m (m = 0, 1, ...): pairs (o, o + NT) per iteration, (b, k)
    // relative to b0 walked incrementally
    const int32_t neg32 = (int32_t)neg, db = NT / neg32, dk = NT - db * neg32;
    int32_t b = tid / neg32, k = tid - b * neg32;
    // a part of at most SL * NT slots (the usual case) keeps its slots' entities and LDS ranks in registers
    // until the bucket bases are known: one store per slot, no reload
    const bool one = o1 - o0 <= (int64_t)SL * NT;
    int32_t keep_e[SL], keep_r[SL];
#pragma unroll
    for (int i = 0; i < SL; ++i) keep_e[i] = keep_r[i] = 0;
    for (int64_t o = o0 + tid; o < o1; o += SL * NT) {
        // SL slots o + i*NT per iteration, their run searches in lock step; a slot past the end draws nothing
        SlotDraw d[SL];
        int32_t bi = b, ki = k;
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            const bool live = o + i * NT < o1;
            d[i] = slot_prepare(pi + 12 * (live ? bi : b), live ? ki : k, E, filter, g, jt, w.dbg);
            if (!live) { d[i].q.l = 0; d[i].q.r = 1; d[i].search = false; }
            bi += db; ki += dk;
            if (ki >= neg32) { ki -= neg32; ++bi; }
        }
        slot_searchN<SL>(d);
#pragma unroll
        for (int i = 0; i < SL; ++i) {
            if (o + i * NT < o1) {
                nrec[o + i * NT] = (int32_t)((d[i].e << 1) | d[i].side);
                const int32_t r = lds_rank<PACK>(cnt, d[i].e);
                if (one) {
                    keep_e[i] = (int32_t)d[i].e;
                    keep_r[i] = r;
                } else {
                    noff[o + i * NT] = r;
                }
            }
        }
        b = bi; k = ki;
    }
    __syncthreads();
    PT_PHASE(2);
    // reserve this part's range in every touched call-wide bucket with one returning atomic per count
    // word (packed: the call's global counts are packed the same way, each half < 65536, so one add
    // reserves both buckets); the LDS word becomes the bases. Batches of 8 words per thread keep the
    // atomics in flight together (a returned value is only waited for at its LDS write).
    int32_t *gcnt = w.cnt + call * w.cnt_stride;
    for (int64_t i0 = tid; i0 < cwords; i0 += 8 * NT) {
        int32_t v[8], r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = i0 + u * NT;
            v[u] = i < cwords ? cnt[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = v[u] ? agent_add(&gcnt[i0 + u * NT], v[u]) : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (v[u]) cnt[i0 + u * NT] = r[u];
    }
    __syncthreads();
    PT_PHASE(3);
    // rank inside the call-wide bucket: from registers, or re-read (same thread, same addresses)
    if (one) {
#pragma unroll
        for (int i = 0; i < SL; ++i)
            if (o0 + tid + i * NT < o1) noff[o0 + tid + i * NT] = keep_r[i] + lds_bucket<PACK>(cnt, keep_e[i]);
    } else {
        for (int64_t o = o0 + tid; o < o1; o += NT) noff[o] += lds_bucket<PACK>(cnt, nrec[o] >> 1);
    }
    // every wave's count atomics have returned (their values were used): count this part done. No fence:
    // everything the parts exchange inside this launch is an agent-scope atomic RMW (count words, tickets,
    // the last part's exchanges), performed at the device's coherence point. A part's count adds have
    // returned before the barrier, so they are performed before its ticket add is issued; the last part's
    // exchanges depend on its ticket's returned value, so they are performed after every other part's
    // ticket and therefore after every count add. The plain stores (slot ranks, starts) are read only by
    // later launches. (Measured on the driver's 20-step chunk: thread 0 fencing around the tickets 2.7 ->
    // 3.4-4.1 us per step, every thread fencing 9.5-11.4 us: each fence writes back the XCD's L2.)
    __syncthreads();
    if (tid == 0) is_last = agent_add(&w.tick[call], 1) == (int32_t)(parts - 1);
    __syncthreads();
    PT_PHASE(4);
    if (prof && tid == 0) prof[7] = is_last;
    if (!is_last) return;
    if (tid == 0) w.tick[call] = 0;   // plain store: read again only by a later launch (kernel boundary)
    // last part: the call's bucket sizes, exchanged with zeros (atomics on both sides: every part's adds
    // are seen, and the counts are clear for the next chunk) into LDS, 8 exchanges in flight per thread
    for (int64_t i0 = tid; i0 < cwords; i0 += 8 * NT) {
        int32_t r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = i0 + u * NT < cwords ? agent_exch(&gcnt[i0 + u * NT], 0) : 0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i0 + u * NT < cwords) cnt[i0 + u * NT] = r[u];
    }
    __syncthreads();
    PT_PHASE(5);
    // exclusive scan over the entities into start[]: contiguous words per thread, wave shuffles, LDS
    // wave totals (k_sample_sort's scan on the packed or plain words)
    int32_t *start = w.start + call * w.start_stride;
    const int64_t per = (cwords + NT - 1) / NT;
    const int64_t lo = tid * per, hi = lo + per < cwords ? lo + per : cwords;
    int32_t tsum = 0;
    for (int64_t i = lo; i < hi; ++i) {
        const int32_t v = cnt[i];
        tsum += PACK ? (v & 0xffff) + (int32_t)((uint32_t)v >> 16) : v;
    }
    int32_t incl = tsum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wtot[wid] = incl;
    __syncthreads();
    int32_t run = incl - tsum;
    for (int q = 0; q < wid; ++q) run += wtot[q];
    for (int64_t i = lo; i < hi; ++i) {
        const int32_t v = cnt[i];
        if constexpr (PACK) {
            start[2 * i] = run;
            run += v & 0xffff;
            if (2 * i + 1 < E) start[2 * i + 1] = run;
            run += (int32_t)((uint32_t)v >> 16);
        } else {
            start[i] = run;
            run += v;
        }
    }
    if (tid == NT - 1) start[E] = run;   // the last thread's chunk ends at the end (or is empty): run = total
    PT_PHASE(6);
#undef PT_PHASE
    // the last call's last part advances the sampler streams past every call's draws: every part of every
    // call read them (positive draws) before its count atomics and tickets
    if (!advance) return;
    __syncthreads();
    if (tid == 0) is_last = agent_add(&w.tick[gridDim.x / parts], 1) == (int32_t)(gridDim.x / parts - 1);
    __syncthreads();
    if (!is_last) return;
    if (tid == 0) w.tick[gridDim.x / parts] = 0;   // plain store: read again only by a later launch
    // plain stores of the advanced states: read only by later launches (every part of this launch read them
    // before its ticket add, which returned before this last part's)
    if (tid < 64) advance_states(states, threads, bs, dpp * (int64_t)(gridDim.x / parts), tid);
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
// One launch pair covers every universe whose dim takes the same lane-group shape (each universe's own dim
// at run time); the pairs' base / normal rows are `ds` floats apart (the largest dim of the launch).
template <int MODEL, int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_lp_bases(const LpUniverseDev *__restrict__ us, const LpPair *__restrict__ pairs,
                                                  int64_t n_pairs, int p_norm, int norm_flag, int64_t ds,
                                                  float *__restrict__ base, float *__restrict__ normal,
                                                  float *__restrict__ tuple_min) {
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
        vstore(nW, normal + pi * ds, D, lane);
    }
    if (norm_flag) vnormalize(A, ah); else ah = A;
#pragma unroll
    for (int k = 0; k < Vec::N; ++k) b.x[k] = pr.side == 0 ? rh.x[k] - ah.x[k] : ah.x[k] + rh.x[k];
    vstore(b, base + pi * ds, D, lane);
}

template <int MODEL, int G, int VEC, int KCH>
__global__ __launch_bounds__(256) void k_lp_scan(const LpUniverseDev *__restrict__ us, const LpPair *__restrict__ pairs,
                                                 const int64_t *__restrict__ uoff, const int32_t *__restrict__ uids,
                                                 int p_norm, int norm_flag, int64_t global_E, int64_t ds,
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
            vload(b, base + pi * ds, D, lane);
            Vec nW;
            if constexpr (MODEL == 1) vload(nW, normal + pi * ds, D, lane);
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

// k_lp_scan_t: the scan transposed - one LANE per entity. A workgroup (4 waves) stages a tile of 64
// consecutive local entity rows in LDS once (row stride D + 1 floats: lane e reading float d of its row hits
// bank (e + d) mod 64, conflict-free), and each wave walks a quarter of the universe's pairs: for a pair, every
// lane sums its own entity's |x + b| (or squares) sequentially over d with the pair's base row uniform across
// the wave - no cross-lane reduction per score - and MINs its score into the key row with one atomic
// instruction for 64 entities, skipped when the row already holds a score no larger (the rows only decrease,
// so a stale read can only make an atomic unnecessary, never wrong). TransE rows are normalized once per
// tile (inverse norm per lane); TransH rows are projected on the pair's normal and normalized per pair.
// sum over d < D of f(d) in 8 interleaved partial sums, combined pairwise: 8 independent add chains per lane
// and a rounding error of order (D / 8 + 3) ulp, near the tree reductions of the lane-group kernels
template <typename F>
__device__ __forceinline__ float sum8(int D, F f) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int d = 0;
    for (; d + 8 <= D; d += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] += f(d + k);
    }
    for (int k = 0; d + k < D; ++k) a[k] += f(d + k);
    return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// acc + |v| as one VOP3 add with the abs source modifier. (Left to itself the compiler packs the adds of two
// partial sums into v_pk_add_f32, which has no abs modifier, and spends a v_and_b32 per term on |v|: 2 VALU
// instructions per term instead of 1.5 with v_pk_fma_f32 + this.)
__device__ __forceinline__ float add_abs(float acc, float v) {
    float r;
    asm("v_add_f32_e64 %0, %1, |%2|" : "=v"(r) : "v"(acc), "v"(v));
    return r;
}

// NP sums of the sum8 form (the same partial sums and combination order for each) over one pass of d: the
// caller's function f(q, d) for sum q reads shared operands (the LDS row) once for all of them. MODE 1: the terms
// are |f(q, d)| (a + |v|, one add); MODE 2: the terms are f(q, d)^2, accumulated by an explicit fma(v, v, a).
// (The TransE scan states every rounding explicitly - an fma where the step is an fma, nothing left to the
// compiler's contraction, which had fused some of a loop's products and not others: the two-pair pass and the
// one-pair remainder of k_lp_scan_t then rounded the same pair's score differently; tests/test_gpu_lp_scan.py.)
template <int NP, int MODE = 0, typename F>
__device__ __forceinline__ void sum8xn(int D, F f, float (&r)[NP]) {
    float a[NP][8];
#pragma unroll
    for (int q = 0; q < NP; ++q)
#pragma unroll
        for (int k = 0; k < 8; ++k) a[q][k] = 0.f;
    int d = 0;
    auto step = [&](float acc, float v) {
        return MODE == 1 ? add_abs(acc, v) : MODE == 2 ? __builtin_fmaf(v, v, acc) : acc + v;
    };
    auto group = [&](int d0) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int q = 0; q < NP; ++q) a[q][k] = step(a[q][k], f(q, d0 + k));
    };
    // (two 8-dim groups per iteration: the next group's operand loads issue before the current group's waits;
    // unrolled by hand - the compiler does not unroll a loop holding the asm add of add_abs)
    for (; d + 16 <= D; d += 16) {
        group(d);
        group(d + 8);
    }
    if (d + 8 <= D) {
        group(d);
        d += 8;
    }
    for (int k = 0; d + k < D; ++k)
#pragma unroll
        for (int q = 0; q < NP; ++q) a[q][k] = step(a[q][k], f(q, d + k));
#pragma unroll
    for (int q = 0; q < NP; ++q)
        r[q] = ((a[q][0] + a[q][1]) + (a[q][2] + a[q][3])) + ((a[q][4] + a[q][5]) + (a[q][6] + a[q][7]));
}

#ifndef PT_LP_PAIRS
#ifndef PT_LP_PAIRS
#define PT_LP_PAIRS 2   // (measured r05, C4 k_lp_scan_t total: 1 pair 137.9 ms, 2 pairs 99.4, 4 pairs 105.3, 8 pairs 128.5)
#endif
#endif

template <int MODEL, int NW>
__global__ __launch_bounds__(64 * NW) void k_lp_scan_t(const LpUniverseDev *__restrict__ us, const LpPair *__restrict__ pairs,
                                                   const int64_t *__restrict__ uoff, const int32_t *__restrict__ uids,
                                                   int p_norm, int norm_flag, int64_t global_E, int64_t ds,
                                                   const float *__restrict__ base, const float *__restrict__ normal,
                                                   float *__restrict__ rows) {
    extern __shared__ float s_x[];   // [64][D + 1]
    // (the wave index made provably uniform: the pair walk, its LpPair records and base rows then live in scalar
    // registers and load through the scalar cache, instead of every lane loading the same base-row words)
    const int lane = (int)threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int32_t u = uids[blockIdx.y];
    const LpUniverseDev U = us[u];
    const int D = (int)U.dim, S = D + 1;
    const int64_t p0 = uoff[2 * u], p1 = uoff[2 * u + 1];
    for (int64_t e0 = (int64_t)blockIdx.x * 64; e0 < U.ent_total; e0 += (int64_t)gridDim.x * 64) {
        const int ne = U.ent_total - e0 < 64 ? (int)(U.ent_total - e0) : 64;
        __syncthreads();   // (the previous tile's readers are done)
        const float *src = U.ent + e0 * D;
        for (int i = (int)threadIdx.x; i < ne * D; i += 64 * NW) {
            const int r = i / D;
            s_x[r * S + (i - r * D)] = src[i];
        }
        __syncthreads();
        const bool live = lane < ne;
        float *xr = s_x + (live ? lane : 0) * S;
        const int64_t col = live ? U.remap[e0 + lane] : 0;
        float inv = 1.f;
        if (MODEL == 0 && norm_flag) {   // F.normalize's scale of this lane's row
            float n2[1];
            sum8xn<1, 2>(D, [&](int, int d) { return xr[d]; }, n2);
            const float n = sqrtf(n2[0]);
            inv = 1.0f / (n > kEps ? n : kEps);
        }
        int64_t pi = p0 + wave;
        if constexpr (MODEL == 0) {
            // TransE: the tile's rows normalized in place once (x * inv: the same rounded products the per-pair form
            // computed), then the wave's pairs PT_LP_PAIRS at a time - pi, pi + NW, ... share every LDS read of the row.
            // Each score keeps its expression and its sum8 order, so the scores are bit-identical to one pair at a time.
            // (the NW waves share the tile: every wave has read it for its norm, then wave 0 normalizes it while the
            // others wait)
            __syncthreads();
            if (wave == 0 && live && norm_flag) {
                for (int d = 0; d < D; ++d) xr[d] = xr[d] * inv;
            }
            __syncthreads();
            constexpr int NPP = PT_LP_PAIRS;   // pairs per pass: pi, pi + NW, ..., pi + NW (NPP - 1)
            for (; pi + NW * (NPP - 1) < p1; pi += NW * NPP) {
                LpPair pr[NPP];
                const float *bq[NPP];
                float sg[NPP], acc[NPP];
                int *cell[NPP];
                int old[NPP];
#pragma unroll
                for (int q = 0; q < NPP; ++q) {
                    pr[q] = pairs[pi + NW * q];
                    bq[q] = base + (pi + NW * q) * ds;
                    sg[q] = pr[q].side == 0 ? 1.f : -1.f;
                    // the key-row cells this pass may lower, read before the sums (their latency hidden behind them)
                    cell[q] = reinterpret_cast<int *>(rows + (int64_t)pr[q].key * global_E + col);
                    old[q] = live ? __builtin_nontemporal_load(cell[q]) : 0;
                }
                if (p_norm == 1)
                    sum8xn<NPP, 1>(D, [&](int q, int d) { return __builtin_fmaf(sg[q], xr[d], bq[q][d]); }, acc);
                else
                    sum8xn<NPP, 2>(D, [&](int q, int d) { return __builtin_fmaf(sg[q], xr[d], bq[q][d]); }, acc);
                if (live) {
#pragma unroll
                    for (int q = 0; q < NPP; ++q) {
                        const float sc = p_norm == 1 ? acc[q] : sqrtf(acc[q]);
                        const int bits = __float_as_int(sc);
                        if (bits < old[q]) atomicMin(cell[q], bits);
                    }
                }
            }
            inv = 1.f;   // (the row is normalized in LDS now)
        }
        for (; pi < p1; pi += NW) {
            const LpPair pr = pairs[pi];
            const float *b = base + pi * ds;
            const float sg = pr.side == 0 ? 1.f : -1.f;   // side 0: x-hat + b; side 1: b - x-hat
            float acc;
            if constexpr (MODEL == 0) {   // (the row is normalized in LDS: inv = 1)
                float a1[1];
                if (p_norm == 1)
                    sum8xn<1, 1>(D, [&](int, int d) { return __builtin_fmaf(sg, xr[d] * inv, b[d]); }, a1);
                else
                    sum8xn<1, 2>(D, [&](int, int d) { return __builtin_fmaf(sg, xr[d] * inv, b[d]); }, a1);
                acc = a1[0];
            } else {
                const float *nw = normal + pi * ds;
                const float xd = sum8(D, [&](int d) { return xr[d] * nw[d]; });
                float sc = 1.f;
                if (norm_flag) {
                    const float n = sqrtf(sum8(D, [&](int d) {
                        const float t = xr[d] - xd * nw[d];
                        return t * t;
                    }));
                    sc = 1.0f / (n > kEps ? n : kEps);
                }
                acc = p_norm == 1 ? sum8(D, [&](int d) { return fabsf(sg * ((xr[d] - xd * nw[d]) * sc) + b[d]); })
                                  : sum8(D, [&](int d) {
                                        const float v = sg * ((xr[d] - xd * nw[d]) * sc) + b[d];
                                        return v * v;
                                    });
            }
            const float score = p_norm == 1 ? acc : sqrtf(acc);
            if (live) {
                int *cell = reinterpret_cast<int *>(rows + (int64_t)pr.key * global_E + col);
                const int bits = __float_as_int(score);
                if (bits < *cell) atomicMin(cell, bits);
            }
        }
    }
}

}  // namespace dev

// ==================================================================== host launchers ===========
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
                         int64_t neg_rel, int mode, int bern, int filter, int64_t *h, int64_t *t, int64_t *r, float *y,
                         hipStream_t st) {
    if (bs <= 0) return hipSuccess;
    const int bl = 256;
    hipLaunchKernelGGL(dev::k_sample, dim3((unsigned)((bs + bl - 1) / bl)), dim3(bl), 0, st, g, states, threads, bs,
                       neg, neg_rel, mode, bern, filter, h, t, r, y);
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

static size_t jump_tab_bytes(int64_t neg) { return 16 * (size_t)(neg < 256 ? neg : 256); }   // kJumpTab
static size_t sample_sort_lds(int64_t bs, int64_t neg, int64_t n) {
    // jump maps + counts + per-positive records
    return jump_tab_bytes(neg) + 4 * (size_t)((n + 3) & ~int64_t(3)) + 48 * (size_t)bs;
}
static const size_t kSampleSortLds = 160 * 1024 - 256;   // leaves room for the static wave totals

bool sample_sort_prepare(int64_t bs, int64_t neg, int64_t n, int64_t start_stride) {
    if (sample_sort_lds(bs, neg, n) > kSampleSortLds || n + 1 > start_stride || n >= (int64_t(1) << 30)) return false;
    return hipFuncSetAttribute(reinterpret_cast<const void *>(dev::k_sample_sort),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSampleSortLds) == hipSuccess;
}

hipError_t launch_sample_sort(const DeviceGraph &g, const uint64_t *states, int64_t threads, int64_t bs, int64_t neg,
                              int bern, int filter, int64_t calls, int64_t n, const CsrWork &w, hipStream_t st) {
    const size_t lds = sample_sort_lds(bs, neg, n);
    if (lds > kSampleSortLds || n + 1 > w.start_stride) return hipErrorInvalidValue;
    hipLaunchKernelGGL(dev::k_sample_sort, dim3((unsigned)calls), dim3(1024), lds, st, g, states, threads, bs, neg,
                       bern, filter, n, w);
    return hipGetLastError();
}

// split sampler: threads per workgroup (PT_PART_NT = 256 | 512 | 1024 for tuning), LDS plan
static int part_nt() {
    static const int nt = [] {
        const char *v = pt_tuning_env("PT_PART_NT");
        const int x = v ? atoi(v) : 512;
        return x == 256 || x == 1024 ? x : 512;
    }();
    return nt;
}
static bool part_pack(int64_t bs, int64_t neg) { return bs * neg < 65536; }
static size_t sample_part_lds(int64_t bs, int64_t neg, int64_t n, int64_t parts) {
    const int64_t cw = part_pack(bs, neg) ? (n + 1) >> 1 : n;
    const int64_t np = (bs + parts - 1) / parts + 1;   // positives of the largest part
    return jump_tab_bytes(neg) + 4 * (size_t)((cw + 3) & ~int64_t(3)) + 48 * (size_t)np;
}

// lock-step slots per thread: 4 when a part holds >= 3 slots per thread, else 2
static int part_sl(int64_t bs, int64_t neg, int64_t parts) {
    const int64_t per = (bs + parts - 1) / parts * neg;
    return per >= 3 * part_nt() ? 4 : 2;
}

template <int NT, bool PACK>
static hipError_t part_attr() {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(dev::k_sample_part<NT, PACK, 2>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSampleSortLds);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute(reinterpret_cast<const void *>(dev::k_sample_part<NT, PACK, 4>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSampleSortLds);
}

bool sample_part_fits(int64_t bs, int64_t neg, int64_t n, int64_t parts) {
    return parts >= 1 && parts <= bs && neg >= 1 && sample_part_lds(bs, neg, n, parts) <= kSampleSortLds &&
           n < (int64_t(1) << 30) && bs * neg < (int64_t(1) << 30);
}

bool sample_part_prepare(int64_t bs, int64_t neg, int64_t n, int64_t parts) {
    if (!sample_part_fits(bs, neg, n, parts)) return false;
    const bool pk = part_pack(bs, neg);
    switch (part_nt()) {
        case 256: return (pk ? part_attr<256, true>() : part_attr<256, false>()) == hipSuccess;
        case 1024: return (pk ? part_attr<1024, true>() : part_attr<1024, false>()) == hipSuccess;
        default: return (pk ? part_attr<512, true>() : part_attr<512, false>()) == hipSuccess;
    }
}

hipError_t launch_sample_part(const DeviceGraph &g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg,
                              int bern, int filter, int64_t calls, int64_t parts, int64_t n, const CsrWork &w,
                              hipStream_t st, int64_t call0, int advance) {
    if (!sample_part_fits(bs, neg, n, parts) || n + 1 > w.start_stride || n > w.cnt_stride || !w.tick)
        return hipErrorInvalidValue;
    const size_t lds = sample_part_lds(bs, neg, n, parts);
    const dim3 grid((unsigned)(calls * parts));
    const bool pk = part_pack(bs, neg);
    const int sl = part_sl(bs, neg, parts);
#define PT_PART(NT_, PK_, SL_)                                                                                 \
    if (part_nt() == NT_ && pk == PK_ && sl == SL_) {                                                        \
        hipLaunchKernelGGL((dev::k_sample_part<NT_, PK_, SL_>), grid, dim3(NT_), lds, st, g, states, threads, \
                           bs, neg, bern, filter, parts, w, call0, advance);                                  \
        return hipGetLastError();                                                                            \
    }
    PT_PART(256, true, 2) PT_PART(256, true, 4) PT_PART(256, false, 2) PT_PART(256, false, 4)
    PT_PART(512, true, 2) PT_PART(512, true, 4) PT_PART(512, false, 2) PT_PART(512, false, 4)
    PT_PART(1024, true, 2) PT_PART(1024, true, 4) PT_PART(1024, false, 2) PT_PART(1024, false, 4)
#undef PT_PART
    return hipErrorInvalidValue;
}

hipError_t launch_scan_counts(const CsrWork &w, int64_t n, int64_t calls, uint64_t *states, int64_t threads,
                              int64_t bs, int64_t dpp, hipStream_t st) {
    hipLaunchKernelGGL(dev::k_scan_counts, dim3((unsigned)calls), dim3(1024), 0, st, w.cnt, w.start, n, states, threads,
                       bs, dpp, w, bs * ((dpp - 1) / 2));
    return hipGetLastError();
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

// PT_LP_SCAN_T (measurement builds): 1 = the transposed scan k_lp_scan_t (default), 0 = k_lp_scan
#ifndef PT_LP_SCAN_T
#define PT_LP_SCAN_T 1
#endif
// k_lp_scan_t's waves per workgroup sharing one tile (PT_LP_WAVES = 4 | 8 | 16 in the tuning build; measured r05,
// C4's nine launches: 4 waves 85.3 ms, 8 waves 77.1 ms, 16 waves 91.3 ms, profiles/r05_c4_lp_waves.json)
static int lp_waves() {
    static const int nw = [] {
        const char *v = pt_tuning_env("PT_LP_WAVES");
        const int x = v ? atoi(v) : 8;
        return x == 4 || x == 16 ? x : 8;
    }();
    return nw;
}
hipError_t launch_lp_min(const LpUniverseDev *us, const LpPair *pairs, int64_t n_pairs, const int64_t *uoff,
                         const int32_t *uids, int64_t n_active, int64_t dim, int64_t max_ent, int model, int p_norm,
                         int norm_flag, int64_t global_E, int64_t ds, float *base, float *normal, float *rows,
                         float *tuple_min, hipStream_t st) {
    if (n_pairs <= 0) return hipSuccess;
    const Shape s = pick_shape(dim);
    // the transposed scan's tile of 64 rows in LDS (row stride dim + 1)
    const size_t lds_t = sizeof(float) * 64 * (size_t)(dim + 1);
    const int nw = lp_waves();
    if (PT_LP_SCAN_T && lds_t > (64 << 10) && lds_t <= (160 << 10)) {
        const void *fn[6] = {reinterpret_cast<const void *>(dev::k_lp_scan_t<0, 4>),
                             reinterpret_cast<const void *>(dev::k_lp_scan_t<1, 4>),
                             reinterpret_cast<const void *>(dev::k_lp_scan_t<0, 8>),
                             reinterpret_cast<const void *>(dev::k_lp_scan_t<1, 8>),
                             reinterpret_cast<const void *>(dev::k_lp_scan_t<0, 16>),
                             reinterpret_cast<const void *>(dev::k_lp_scan_t<1, 16>)};
        const int k = nw == 4 ? 0 : nw == 8 ? 2 : 4;
        for (int m = 0; m < 2; ++m) {
            const hipError_t e = hipFuncSetAttribute(fn[k + m], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_t);
            if (e != hipSuccess) return e;
        }
    }
    const int64_t gpb = 256 / s.G;
    const dim3 gb((unsigned)((n_pairs + gpb - 1) / gpb)), block(256);
    int64_t bx = (max_ent + gpb * 4 - 1) / (gpb * 4);
    if (bx > 32) bx = 32;
    if (bx < 1) bx = 1;
#define PT_LPT(NW_)                                                                                                \
    if (nw == NW_) {                                                                                               \
        if (model == 0)                                                                                            \
            hipLaunchKernelGGL((dev::k_lp_scan_t<0, NW_>), gt, bt, lds_t, st, us, pairs, uoff, uids + y0, p_norm,    \
                               norm_flag, global_E, ds, base, normal, rows);                                       \
        else                                                                                                       \
            hipLaunchKernelGGL((dev::k_lp_scan_t<1, NW_>), gt, bt, lds_t, st, us, pairs, uoff, uids + y0, p_norm,    \
                               norm_flag, global_E, ds, base, normal, rows);                                       \
    }
#define PT_LP(G_, V_, K_)                                                                                          \
    if (s.G == G_ && s.VEC == V_ && s.KCH == K_) {                                                               \
        for (int64_t y0 = 0; y0 < n_active; y0 += 65535) {                                                         \
            const dim3 gs((unsigned)bx, (unsigned)(n_active - y0 < 65535 ? n_active - y0 : 65535));              \
            if (y0 == 0) {                                                                                         \
                if (model == 0)                                                                                    \
                    hipLaunchKernelGGL((dev::k_lp_bases<0, G_, V_, K_>), gb, block, 0, st, us, pairs, n_pairs,    \
                                       p_norm, norm_flag, ds, base, normal, tuple_min);                            \
                else                                                                                               \
                    hipLaunchKernelGGL((dev::k_lp_bases<1, G_, V_, K_>), gb, block, 0, st, us, pairs, n_pairs,    \
                                       p_norm, norm_flag, ds, base, normal, tuple_min);                            \
            }                                                                                                      \
            if (PT_LP_SCAN_T && lds_t <= (160 << 10)) {                                                         \
                const dim3 gt((unsigned)((max_ent + 63) / 64), gs.y), bt((unsigned)(64 * nw));                   \
                PT_LPT(4) PT_LPT(8) PT_LPT(16)                                                                     \
            } else if (model == 0)                                                                                 \
                hipLaunchKernelGGL((dev::k_lp_scan<0, G_, V_, K_>), gs, block, 0, st, us, pairs, uoff, uids + y0,   \
                                   p_norm, norm_flag, global_E, ds, base, normal, rows);                            \
            else                                                                                                   \
                hipLaunchKernelGGL((dev::k_lp_scan<1, G_, V_, K_>), gs, block, 0, st, us, pairs, uoff, uids + y0,   \
                                   p_norm, norm_flag, global_E, ds, base, normal, rows);                            \
        }                                                                                                          \
        return hipGetLastError();                                                                                  \
    }
    PT_SHAPES(PT_LP)
#undef PT_LP
#undef PT_LPT
    return hipErrorInvalidValue;
}

}  // namespace pt
