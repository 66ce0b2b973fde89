// Host-side launch interface of the HIP kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "graph.h"

namespace pt {

struct StepParams {
    int model, p_norm, norm_flag, opt;
    float lr, margin;
    int64_t ent_total, rel_total, dim;
    float *ent, *rel, *normv;
    float *ent_acc, *rel_acc, *norm_acc;
    int64_t batch_size, neg;
    float inv_count;   // 1 / (batch_size * neg)
    int loss_assign = 0;   // the apply pass stores the step's loss (=) instead of adding it (+=)
    int dbg = 0;       // timing experiments only (PT_STEP_DBG): bit 0 skip corrupted-row stores, bit 1 skip
                       // positive-row atomics, bit 2 skip negative row loads (results are then wrong)
};

struct StepWorkspace {
    float *gent = nullptr, *grel = nullptr, *gnorm = nullptr;   // gradient rows (zero between steps)
    int *fent = nullptr, *frel = nullptr, *fnorm = nullptr;      // touched-row flags
    // per-positive loss partials [batch]: sum over the positive's negatives of max(p - n, -m); the apply
    // pass reduces them in a fixed order into the step's loss (one same-address float atomic per
    // positive serialises at the memory side: it cost ~13 us per C2 step)
    float *lpart = nullptr;
};

// Workspace of the counting-sort (CSR) gradient path for large neg (see k_sample_csr). The sampling
// and scan passes fill `calls` consecutive steps at once (pos/neg/off/cnt/start are [calls][...]);
// a per-step view (csr_view) offsets the pointers to one step.
struct CsrWork {
    int4 *pos = nullptr;        // [calls][bs] (h, r, t, -)
    int32_t *neg = nullptr;     // [calls][bs*neg] entity << 1 | tail_side
    int32_t *off = nullptr;     // [calls][bs*neg] destination row of the slot in the counting-sort order
                                // (rank_only: its rank inside the entity's bucket; the step adds start[e])
    int32_t *cnt = nullptr;     // [calls][cnt_stride] bucket sizes (zero between uses)
    int32_t *start = nullptr;   // [calls][start_stride] exclusive prefix of cnt (E+1 used)
    float *contrib = nullptr;   // [bs*neg][dim] gradient rows of the corrupted entities (one step)
    int32_t *tick = nullptr;    // [calls + 1] parts of a call done, then calls done (k_sample_part; zero
                                // between uses)
    int rank_only = 0;          // off[] holds bucket ranks (k_sample_part) instead of destinations
    uint64_t *prof = nullptr;   // PT_PART_PROF=1 only: [workgroup][8] phase timestamps of k_sample_part
    int dbg = 0;                // timing experiments only (PT_PART_DBG; results then wrong): bit 0 no run
                                // search, bit 1 no stream jump, bit 2 no 64-bit modulo
    int64_t cnt_stride = 0, start_stride = 0;
    // fused step + apply (step_apply.hip): per call, the positives' uses of every table row - entity rows
    // [0, E) as h or t, relation rows [rel_base, rel_base + R) - counted by the sampler ([calls][use_stride],
    // zeroed before each chunk's sampling); per call the positives' loss partials ([calls][bs])
    int32_t *uses = nullptr;
    int64_t use_stride = 0, rel_base = 0;
    float *lpart = nullptr;
    // slot-scale mode (pt_trainer_set_slot_scale, k_step_csr + k_apply_buf): instead of a corrupted entity's
    // gradient row, the step stores per slot (at its counting-sort destination) the positive (b << 1 | tail side)
    // and the scalar k of d loss / d v = k v (p = 2) or k sign(v) (p = 1), plus per positive its normalized rows
    // (h-hat + r-hat, r-hat, t-hat) in `bases` ([bs][3][dim]); the apply pass re-forms each slot's row from them
    // and the entity's own row - the same operations, so the same bits - in bucket order. srec and bases live in
    // the contrib region (one step).
    int slot_scale = 0;
    int2 *srec = nullptr;
    float *bases = nullptr;
};

inline CsrWork csr_view(const CsrWork &w, int64_t call, int64_t bs, int64_t neg) {
    CsrWork v = w;
    v.pos = w.pos + call * bs;
    v.neg = w.neg + call * bs * neg;
    v.off = w.off + call * bs * neg;
    v.cnt = w.cnt + call * w.cnt_stride;
    v.start = w.start + call * w.start_stride;
    if (w.uses) v.uses = w.uses + call * w.use_stride;
    if (w.lpart) v.lpart = w.lpart + call * bs;
    return v;
}

struct LpUniverseDev {
    const float *ent, *rel, *normv;
    const int64_t *remap;   // local -> global entity
    int64_t ent_total, dim;
};

struct LpPair {
    int32_t key, universe, anchor, rel, side;   // local anchor entity / relation ids
};

// lane-group shape of a row of D floats: G lanes x KCH chunks of VEC floats (kernels.hip header)
struct Shape {
    int G, VEC, KCH;
};

inline Shape pick_shape(int64_t D, bool vec4 = true) {
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

// instantiated (G, VEC, KCH) row shapes
#define PT_SHAPES(X)                                                                                  \
    X(2, 4, 1) X(4, 4, 1) X(8, 4, 1) X(16, 4, 1) X(32, 4, 1) X(64, 4, 1) X(64, 4, 2)                 \
    X(2, 1, 1) X(4, 1, 1) X(8, 1, 1) X(16, 1, 1) X(32, 1, 1) X(64, 1, 1) X(64, 1, 2) X(64, 1, 4)    \
    X(64, 1, 8)

bool shape_supported(int64_t dim);
hipError_t launch_sample(const DeviceGraph &g, const uint64_t *states, int64_t threads, int64_t bs, int64_t neg,
                         int64_t neg_rel, int mode, int bern, int filter, int64_t *h, int64_t *t, int64_t *r, float *y,
                         hipStream_t st);
hipError_t launch_spin(int64_t us, hipStream_t st);
hipError_t launch_advance(uint64_t *states, int64_t threads, int64_t bs, int64_t dpp, hipStream_t st);
hipError_t launch_sample_csr(const DeviceGraph &g, const uint64_t *states, int64_t threads, int64_t bs, int64_t neg,
                             int bern, int filter, int64_t calls, const CsrWork &w, hipStream_t st);
// one workgroup per call: sampling + LDS counting sort + scan; the streams are NOT advanced (launch_advance).
// sample_sort_prepare: whether the LDS plan fits for (bs, neg, n) (and the kernel's LDS limit is raised);
// otherwise use launch_sample_csr + launch_scan_counts
bool sample_sort_prepare(int64_t bs, int64_t neg, int64_t n, int64_t start_stride);
hipError_t launch_sample_sort(const DeviceGraph &g, const uint64_t *states, int64_t threads, int64_t bs, int64_t neg,
                              int bern, int filter, int64_t calls, int64_t n, const CsrWork &w, hipStream_t st);
// `parts` workgroups per call: sampling + LDS counting sort of each part, call-wide buckets reserved with
// one atomic per touched count word, the last part of a call scans, the last call advances the streams;
// off[] holds bucket ranks (the caller sets CsrWork::rank_only for the step kernels).
// sample_part_fits: whether the LDS plan of `parts` parts per call fits; sample_part_prepare: the same,
// and raises the kernel's LDS limit (call outside any stream capture)
bool sample_part_fits(int64_t bs, int64_t neg, int64_t n, int64_t parts);
bool sample_part_prepare(int64_t bs, int64_t neg, int64_t n, int64_t parts);
hipError_t launch_sample_part(const DeviceGraph &g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg,
                              int bern, int filter, int64_t calls, int64_t parts, int64_t n, const CsrWork &w,
                              hipStream_t st, int64_t call0 = 0, int advance = 1);
hipError_t launch_scan_counts(const CsrWork &w, int64_t n, int64_t calls, uint64_t *states, int64_t threads,
                              int64_t bs, int64_t dpp, hipStream_t st);
bool step_fits(const StepParams &P, int64_t neg, bool csr);
hipError_t launch_step(const StepParams &P, const DeviceGraph &g, const uint64_t *states, int64_t threads, int bern,
                       int filter, const int64_t *bh, const int64_t *bt, const int64_t *br, const StepWorkspace &W,
                       float *loss, hipStream_t st, const CsrWork *csr = nullptr);
hipError_t launch_apply(const StepParams &P, const StepWorkspace &W, uint64_t *states, int64_t threads, int64_t bs,
                        int64_t dpp, float *loss, hipStream_t st, const CsrWork *csr = nullptr);
hipError_t launch_score(const StepParams &P, int mode, const int64_t *h, const int64_t *t, const int64_t *r, int64_t n,
                        float *out, hipStream_t st);
hipError_t launch_score_queries(const StepParams &P, int side, const int64_t *qh, const int64_t *qt, const int64_t *qr,
                                int64_t nq, int64_t E, float *out, hipStream_t st, int global_order = 0);
// pairs sorted by universe; universe u's pairs are pairs[uoff[2u] .. uoff[2u+1]); uids = the n_active
// universes with pairs, all of dims that take dim's lane-group shape (pick_shape); base / normal: scratch
// [n_pairs][ds], ds >= every such dim
hipError_t launch_lp_min(const LpUniverseDev *us, const LpPair *pairs, int64_t n_pairs, const int64_t *uoff,
                         const int32_t *uids, int64_t n_active, int64_t dim, int64_t max_ent, int model, int p_norm,
                         int norm_flag, int64_t global_E, int64_t ds, float *base, float *normal, float *rows,
                         float *tuple_min, hipStream_t st);

hipError_t launch_torch_init(const pt_torch_init_job *d_jobs, int64_t n, hipStream_t st);
hipError_t launch_rank_rows(const float *rows, int64_t E, const int64_t *row_of, const int64_t *truth,
                            const float *repl, const int64_t *part_off, const int64_t *part, int64_t nq, int64_t *raw,
                            int64_t *filt, hipStream_t st);
hipError_t launch_rank_types(const float *rows, int64_t E, const int64_t *row_of, const int64_t *truth,
                             const float *repl, const int64_t *rel, const int64_t *type_lef, const int64_t *type_rig,
                             const int64_t *types, const int64_t *part_off, const int64_t *part, int64_t nq,
                             int64_t *raw, int64_t *filt, hipStream_t st);

}  // namespace pt
