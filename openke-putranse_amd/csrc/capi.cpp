// C-ABI of libputranse_hip.so (include/putranse.h): reentrant pt_* entry points and the reference's
// Base.so symbols for the hot path, all executing batch construction / training / scoring on the GPU.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <tuple>
#include <queue>
#include <set>
#include <unordered_map>
#include <vector>

#include "tuning.h"
#include "common.h"
#include "graph.h"
#include "kernels.h"
#include "ordered.h"
#include "rng.h"
#include "step_apply.h"
#include "universe.h"
#include "universes.h"

// ======================================================================== errors =================
namespace pt {
namespace {
thread_local std::string g_err;
}
void set_error(int code, const std::string &msg) { g_err = "[putranse error " + std::to_string(code) + "] " + msg; }
int fail(int code, const std::string &msg) {
    set_error(code, msg);
    return code;
}
}  // namespace pt

extern "C" const char *pt_last_error(void) { return pt::g_err.c_str(); }
extern "C" int pt_version(void) { return 1; }

// ======================================================================== objects ================
struct pt_sampler {
    pt::Graph *g = nullptr;        // graph sampled from (follows swaps for the legacy context)
    int64_t threads = 0;
    uint64_t *d_states = nullptr;  // device LCG states, one per emulated sampler thread
    int device = -1;
    ~pt_sampler() {
        if (d_states) (void)hipFree(d_states);
    }
};

struct GraphKey {
    const void *sampler, *graph, *losses, *states;
    int64_t bs, neg, bern, filter, steps;
    bool operator<(const GraphKey &o) const {
        return std::tie(sampler, graph, losses, states, bs, neg, bern, filter, steps) <
               std::tie(o.sampler, o.graph, o.losses, o.states, o.bs, o.neg, o.bern, o.filter, o.steps);
    }
};

struct pt_trainer {
    pt::StepParams P{};
    pt::StepWorkspace W{};
    void *ws_block = nullptr;
    size_t ws_bytes = 0;   // gradient rows + touched flags (all zero between steps)
    // counting-sort gradient path for large neg (allocated on first use, grown as needed)
    void *csr_block = nullptr;
    size_t csr_cap = 0;
    pt::CsrWork csr{};
    int64_t csr_bs = 0, csr_neg = 0, csr_chunk = 0;   // layout the workspace was carved for
    bool csr_fused = false;                             // k_sample_sort plan fits LDS
    // the fused step + apply (step_apply.hip) for TransE with 33-256 float4 chunks per row: its rows and
    // arrival words live in the counting-sort workspace (fr.gent == nullptr: not carved for it)
    pt::FusedRows fr{};
    bool step_apply_on = false;                         // pt_trainer_set_step_apply (opt-in: measured slower)
    bool slot_scale_on = false;                         // pt_trainer_set_slot_scale (CsrWork::slot_scale)
    bool last_step_apply = false;                       // the last enqueued in-kernel-sampled steps took it
    bool csr_part = false;                              // k_sample_part prepared (its LDS limit raised)
    int last_path = -1;                                 // sampling path of the last enqueued chunk (PT_PATH_*)
    int64_t lpart_cap = 0;                             // W.lpart capacity (positives)
    int device = -1;
    hipStream_t cap = nullptr;
    // the split sampler's second launch of a chunk (sample_split_head): its stream and the fork / join events
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int64_t split_override = -1;                        // pt_trainer_set_sample_split: head steps, 0 off, -1 auto
    std::map<GraphKey, hipGraphExec_t> graphs;
    int path_override = -1;                             // pt_trainer_set_sampling: PT_PATH_* or -1 (automatic)
    int64_t parts_override = 0;                         // split-sampler workgroups per call (0: automatic)
    int64_t prof_calls = 0, prof_parts = 0, prof_cap = 0;   // PT_PART_PROF (tuning build) record layout
    // reference-order (deterministic) mode: ordered.hip's step on k_sample batches (pt_trainer_set_deterministic)
    bool ordered = false;
    void *ord_block = nullptr;
    size_t ord_cap = 0;
    int64_t *ord_h = nullptr, *ord_t = nullptr, *ord_r = nullptr;
    float *ord_y = nullptr, *ord_score = nullptr, *ord_ds = nullptr;
    float *ord_g = nullptr;   // [4][seq][dim] per-slot gradient rows
    void drop_graphs() {
        for (auto &kv : graphs) (void)hipGraphExecDestroy(kv.second);
        graphs.clear();
    }
    ~pt_trainer() {
        drop_graphs();
        if (cap) (void)hipStreamDestroy(cap);
        if (side) (void)hipStreamDestroy(side);
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);

        if (ws_block) (void)hipFree(ws_block);
        if (csr_block) (void)hipFree(csr_block);
        if (csr.prof) (void)hipFree(csr.prof);
        if (W.lpart) (void)hipFree(W.lpart);
        if (ord_block) (void)hipFree(ord_block);
    }
};

namespace {

int desc_to_params(const pt_model_desc *m, pt::StepParams &P) {
    PT_CHECK(m, PT_EINVAL, "null model descriptor");
    PT_CHECK(m->model == PT_TRANSE || m->model == PT_TRANSH, PT_EINVAL, "model must be PT_TRANSE or PT_TRANSH");
    PT_CHECK(m->p_norm == 1 || m->p_norm == 2, PT_ENOTSUP, "p_norm must be 1 or 2");
    PT_CHECK(m->opt == PT_SGD || m->opt == PT_ADAGRAD, PT_EINVAL, "opt must be PT_SGD or PT_ADAGRAD");
    PT_CHECK(pt::shape_supported(m->dim), PT_ENOTSUP, "embedding dim " + std::to_string(m->dim) + " not supported");
    PT_CHECK(m->ent && m->rel && m->ent_total > 0 && m->rel_total > 0, PT_EINVAL, "missing tables");
    PT_CHECK(m->model == PT_TRANSE || m->normv, PT_EINVAL, "TransH needs norm_vector");
    PT_CHECK(m->opt == PT_SGD || (m->ent_acc && m->rel_acc && (m->model == PT_TRANSE || m->norm_acc)), PT_EINVAL,
             "Adagrad needs state_sum buffers");
    P.model = m->model;
    P.p_norm = m->p_norm;
    P.norm_flag = m->norm_flag ? 1 : 0;
    P.opt = m->opt;
    P.lr = m->lr;
    P.margin = m->margin;
    P.ent_total = m->ent_total;
    P.rel_total = m->rel_total;
    P.dim = m->dim;
    P.ent = m->ent; P.rel = m->rel; P.normv = m->normv;
    P.ent_acc = m->ent_acc; P.rel_acc = m->rel_acc; P.norm_acc = m->norm_acc;
    if (const char *v = pt_tuning_env("PT_STEP_DBG")) P.dbg = atoi(v);
    return PT_OK;
}

// negatives at or above this count take the counting-sort path (PT_CSR=0/1 overrides)
bool use_csr(int64_t neg) {
    static int forced = [] {
        const char *v = pt_tuning_env("PT_CSR");
        return v ? atoi(v) : -1;
    }();
    return forced >= 0 ? forced != 0 : neg >= 4;
}

int check_step_args(const pt::StepParams &P, pt_sampler *s, int64_t bs, int64_t neg, const int64_t *bh) {
    PT_CHECK(bs > 0 && neg > 0, PT_EINVAL, "batch_size and neg_ent must be positive");
    if (!bh) {
        PT_CHECK(s && s->g && s->d_states, PT_ESTATE, "in-kernel sampling needs a sampler bound to a graph");
        PT_CHECK(s->g->ent_total <= P.ent_total && s->g->rel_total <= P.rel_total, PT_EINVAL,
                 "graph ids exceed the model tables");
        PT_CHECK(s->g->ent_total > 1, PT_EINVAL, "graph needs at least two entities");
        pt::StepParams Q = P;
        Q.batch_size = bs;
        PT_CHECK(pt::step_fits(Q, neg, use_csr(neg)), PT_ENOTSUP, "neg_ent too large for the LDS draw buffer");
    }
    return PT_OK;
}

}  // namespace

// ======================================================================== graphs =================
// Opt-in count-header record format for every *2id.txt reader (pt_graph_load, importTrainFiles,
// importTestFiles); the default keeps the reference's line-count contract (Reader.h:176-196).
extern "C" int pt_set_count_header(int on) {
    pt::set_count_header(on != 0);
    return PT_OK;
}
extern "C" int pt_get_count_header(void) { return pt::count_header() ? 1 : 0; }

extern "C" int pt_graph_load(const char *in_path, pt_graph **out) {
    PT_CHECK(in_path && out, PT_EINVAL, "pt_graph_load: null argument");
    auto *g = new pt_graph();
    int rc = pt::load_graph(in_path, g->g);
    if (rc) {
        delete g;
        return rc;
    }
    *out = g;
    return PT_OK;
}
extern "C" int pt_graph_free(pt_graph *g) {
    delete g;
    return PT_OK;
}
extern "C" int64_t pt_graph_ent_total(const pt_graph *g) { return g ? g->g.ent_total : -1; }
extern "C" int64_t pt_graph_rel_total(const pt_graph *g) { return g ? g->g.rel_total : -1; }
extern "C" int64_t pt_graph_train_total(const pt_graph *g) { return g ? g->g.train_total : -1; }
extern "C" int pt_graph_triples(const pt_graph *g, int64_t *h, int64_t *t, int64_t *r) {
    PT_CHECK(g && h && t && r, PT_EINVAL, "pt_graph_triples: null argument");
    for (int64_t i = 0; i < g->g.train_total; ++i) {
        h[i] = g->g.list[i].h;
        t[i] = g->g.list[i].t;
        r[i] = g->g.list[i].r;
    }
    return PT_OK;
}

// ======================================================================== sampler ================
static int sampler_init(pt_sampler *s, pt::Graph *g, int64_t threads, const uint64_t *seeds) {
    PT_CHECK(threads > 0 && threads <= 64, PT_ENOTSUP, "threads must be in [1, 64]");
    PT_HIP(hipGetDevice(&s->device));
    s->g = g;
    s->threads = threads;
    if (g) {
        int rc = g->upload();
        if (rc) return rc;
    }
    PT_HIP(hipMalloc(&s->d_states, sizeof(uint64_t) * 64));
    PT_HIP(hipMemset(s->d_states, 0, sizeof(uint64_t) * 64));
    if (seeds) PT_HIP(hipMemcpy(s->d_states, seeds, sizeof(uint64_t) * (size_t)threads, hipMemcpyHostToDevice));
    return PT_OK;
}

extern "C" int pt_sampler_create(pt_graph *g, int64_t threads, const uint64_t *seeds, pt_sampler **out) {
    PT_CHECK(g && out && seeds, PT_EINVAL, "pt_sampler_create: null argument");
    auto *s = new pt_sampler();
    int rc = sampler_init(s, &g->g, threads, seeds);
    if (rc) {
        delete s;
        return rc;
    }
    *out = s;
    return PT_OK;
}
extern "C" int pt_sampler_free(pt_sampler *s) {
    delete s;
    return PT_OK;
}
extern "C" int pt_sampler_set_seeds(pt_sampler *s, const uint64_t *seeds) {
    PT_CHECK(s && seeds, PT_EINVAL, "pt_sampler_set_seeds: null argument");
    PT_HIP(hipMemcpy(s->d_states, seeds, sizeof(uint64_t) * (size_t)s->threads, hipMemcpyHostToDevice));
    return PT_OK;
}
extern "C" int pt_sampler_get_seeds(pt_sampler *s, uint64_t *seeds) {
    PT_CHECK(s && seeds, PT_EINVAL, "pt_sampler_get_seeds: null argument");
    PT_HIP(hipMemcpy(seeds, s->d_states, sizeof(uint64_t) * (size_t)s->threads, hipMemcpyDeviceToHost));
    return PT_OK;
}
extern "C" int pt_sampler_sample_ex(pt_sampler *s, int64_t bs, int64_t neg, int64_t neg_rel, int64_t mode,
                                    int64_t bern, int64_t filter, int64_t *d_h, int64_t *d_t, int64_t *d_r, float *d_y,
                                    void *stream) {
    PT_CHECK(s && s->g && d_h && d_t && d_r, PT_EINVAL, "pt_sampler_sample: null argument");
    PT_CHECK(bs >= 0 && neg >= 0 && neg_rel >= 0, PT_EINVAL, "negative batch size or negative rate");
    PT_CHECK(mode >= -1 && mode <= 1, PT_EINVAL, "sampling mode must be 0, -1 (head_batch) or 1 (tail_batch)");
    PT_CHECK(s->g->ent_total > 1, PT_EINVAL, "graph needs at least two entities");
    int rc = s->g->upload();
    if (rc) return rc;
    PT_CHECK(neg_rel == 0 || !s->g->ht_full, PT_EINVAL,
             "corrupt_rel: an (h,t) pair is linked by every relation (the reference divides by zero, Corrupt.h:135)");
    hipStream_t st = (hipStream_t)stream;
    PT_HIP(pt::launch_sample(s->g->dev, s->d_states, s->threads, bs, neg, neg_rel, (int)mode, (int)bern, (int)filter,
                             d_h, d_t, d_r, d_y, st));
    PT_HIP(pt::launch_advance(s->d_states, s->threads, bs, 1 + (mode == 0 ? 2 : 1) * neg + neg_rel, st));
    return PT_OK;
}

extern "C" int pt_sampler_sample(pt_sampler *s, int64_t bs, int64_t neg, int64_t bern, int64_t filter, int64_t *d_h,
                                 int64_t *d_t, int64_t *d_r, float *d_y, void *stream) {
    return pt_sampler_sample_ex(s, bs, neg, 0, 0, bern, filter, d_h, d_t, d_r, d_y, stream);
}

// ======================================================================== training ===============
extern "C" int pt_trainer_create(const pt_model_desc *m, pt_trainer **out) {
    PT_CHECK(out, PT_EINVAL, "pt_trainer_create: null argument");
    auto t = std::make_unique<pt_trainer>();
    int rc = desc_to_params(m, t->P);
    if (rc) return rc;
    PT_HIP(hipGetDevice(&t->device));
    const int64_t E = t->P.ent_total, R = t->P.rel_total, D = t->P.dim;
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t ge = al(4 * E * D), gr = al(4 * R * D), gn = m->model == PT_TRANSH ? al(4 * R * D) : 0;
    const size_t fe = al(4 * E), fr = al(4 * R), fn = m->model == PT_TRANSH ? al(4 * R) : 0;
    const size_t total = ge + gr + gn + fe + fr + fn;
    PT_HIP(hipMalloc(&t->ws_block, total));
    PT_HIP(hipMemset(t->ws_block, 0, total));
    t->ws_bytes = total;
    char *b = (char *)t->ws_block;
    t->W.gent = (float *)b; b += ge;
    t->W.grel = (float *)b; b += gr;
    t->W.gnorm = gn ? (float *)b : nullptr; b += gn;
    t->W.fent = (int *)b; b += fe;
    t->W.frel = (int *)b; b += fr;
    t->W.fnorm = fn ? (int *)b : nullptr;
    PT_HIP(hipStreamCreateWithFlags(&t->cap, hipStreamNonBlocking));
    PT_HIP(hipStreamCreateWithFlags(&t->side, hipStreamNonBlocking));
    PT_HIP(hipEventCreateWithFlags(&t->ev_fork, hipEventDisableTiming));
    PT_HIP(hipEventCreateWithFlags(&t->ev_join, hipEventDisableTiming));
    *out = t.release();
    return PT_OK;
}
extern "C" int pt_trainer_free(pt_trainer *t) {
    delete t;
    return PT_OK;
}
extern "C" int pt_trainer_update_desc(pt_trainer *t, const pt_model_desc *m) {
    PT_CHECK(t, PT_EINVAL, "null trainer");
    pt::StepParams P{};
    int rc = desc_to_params(m, P);
    if (rc) return rc;
    PT_CHECK(P.model == t->P.model && P.ent_total <= t->P.ent_total && P.rel_total <= t->P.rel_total &&
                 P.dim == t->P.dim,
             PT_EINVAL, "descriptor shape differs from the trainer's workspace");
    t->P = P;
    t->drop_graphs();
    return PT_OK;
}


static const int64_t kCsrChunk = 256;   // steps pre-sampled per sampling/scan launch pair
// the fused sampling kernel runs one workgroup per call (~200 us each at C2, latency-bound draws), so it
// only beats the split form once a chunk fills enough CUs on its own
static const int64_t kSampleSortMinCalls = 96;
// the split sampler (k_sample_part) runs ceil(kPartTarget / calls) workgroups per call
static const int64_t kPartTarget = 512;

// Sampling path for a chunk of `calls` steps: pt_trainer_set_sampling forces one (where its plan fits;
// the tuning build also reads PT_SAMPLE_MODE = fused | part | twopass and PT_SAMPLE_TWO_PASS=1); by default
// the fused kernel for chunks of >= kSampleSortMinCalls steps, the split sampler below that.
static int sample_mode(const pt_trainer *t) {
    if (t->path_override >= 0) return t->path_override;
    const char *tp = pt_tuning_env("PT_SAMPLE_TWO_PASS");
    if (tp && atoi(tp) != 0) return PT_PATH_TWO_PASS;
    const char *v = pt_tuning_env("PT_SAMPLE_MODE");
    if (!v) return -1;
    if (!strcmp(v, "fused")) return PT_PATH_FUSED;
    if (!strcmp(v, "part")) return PT_PATH_PART;
    if (!strcmp(v, "twopass")) return PT_PATH_TWO_PASS;
    return -1;
}
static int64_t part_count(const pt_trainer *t, int64_t calls, int64_t bs) {
    int64_t p = (kPartTarget + calls - 1) / calls;
    if (t->parts_override > 0) p = t->parts_override;
    else if (const char *v = pt_tuning_env("PT_PART_COUNT")) p = atoll(v);
    if (p < 2) p = 2;
    return p > bs ? bs : p;
}
static int choose_path(const pt_trainer *t, int64_t calls, int64_t bs, int64_t neg, int forced) {
    const bool part_ok = t->csr_part && pt::sample_part_fits(bs, neg, t->P.ent_total, part_count(t, calls, bs));
    if (forced == PT_PATH_FUSED && t->csr_fused) return PT_PATH_FUSED;
    if (forced == PT_PATH_PART && part_ok) return PT_PATH_PART;
    if (forced == PT_PATH_TWO_PASS) return PT_PATH_TWO_PASS;
    if (t->csr_fused && calls >= kSampleSortMinCalls) return PT_PATH_FUSED;
    if (part_ok) return PT_PATH_PART;
    return PT_PATH_TWO_PASS;
}

// whether the fused step + apply is wanted for this trainer (opt-in, pt_trainer_set_step_apply; the tuning build's
// PT_STEP_APPLY=0 vetoes it): only then does ensure_csr carve its extra state
static bool step_apply_wanted(const pt_trainer *t) {
    static const int forced = [] {
        const char *v = pt_tuning_env("PT_STEP_APPLY");
        return v ? atoi(v) : -1;
    }();
    return t->step_apply_on && forced != 0;
}

// whether the slot-scale mode is wanted (pt_trainer_set_slot_scale; the tuning build's PT_SLOT_SCALE forces it)
static bool slot_scale_wanted(const pt_trainer *t) {
    static const int forced = [] {
        const char *v = pt_tuning_env("PT_SLOT_SCALE");
        return v ? atoi(v) : -1;
    }();
    return forced >= 0 ? forced != 0 : t->slot_scale_on;
}

// Workspace of the counting-sort path, carved once per (bs, neg): room for a chunk of pre-sampled
// steps (<= kCsrChunk, fewer when a step's arrays are large) plus one step's gradient rows. A new
// (bs, neg) re-carves it (and drops captured graphs, whose kernels hold the old pointers).
static int ensure_csr(pt_trainer *t, int64_t bs, int64_t neg) {
    if (t->csr_block && t->csr_bs == bs && t->csr_neg == neg) return PT_OK;
    const int64_t E = t->P.ent_total, R = t->P.rel_total, D = t->P.dim;
    const int64_t cs = (E + 3) & ~int64_t(3), ss = (E + 4) & ~int64_t(3);
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    // the fused step + apply's extra state: per call the rows' uses and the loss partials; padded gradient
    // rows and arrival words; contribution rows at the padded stride
    pt::StepParams Q = t->P;
    Q.batch_size = bs;
    Q.neg = neg;
    const bool sa = step_apply_wanted(t) && pt::step_apply_supported(Q, bs, neg);
    const int64_t dp = sa ? pt::step_apply_row_stride(D) : D, us = (E + R + 63) & ~int64_t(63);
    const size_t per_call = 16 * bs + 8 * bs * neg + 4 * cs + 4 * ss + 4 + 1024 + (sa ? 4 * us + 4 * bs : 0);
    int64_t chunk = (int64_t)std::max<size_t>(1, ((size_t)512 << 20) / per_call);
    chunk = std::min(chunk, kCsrChunk);
    const size_t a_use = sa ? al(4 * us * chunk) : 0, a_lp = sa ? al(4 * bs * chunk) : 0,
                 a_gent = sa ? al(4 * E * dp) : 0, a_grel = sa ? al(4 * R * dp) : 0, a_arr = sa ? al(8 * (E + R)) : 0;
    // slot-scale mode: the step's slot records and positive base rows take the contribution region's place
    // (TransE float4 rows: the k_step_csr / k_apply_buf pair; not with the fused step + apply)
    const bool scm = slot_scale_wanted(t) && !sa && t->P.model == 0 && D % 4 == 0;
    const size_t a_srec = al(8 * bs * neg), a_bases = al(4 * bs * 3 * D);
    const size_t a_pos = al(16 * bs * chunk), a_neg = al(4 * bs * neg * chunk), a_off = a_neg,
                 a_cnt = al(4 * cs * chunk), a_start = al(4 * ss * chunk), a_tick = al(4 * chunk + 4),
                 a_con = std::max(al(4 * bs * neg * dp), scm ? a_srec + a_bases : (size_t)0);
    const size_t need = a_use + a_lp + a_gent + a_grel + a_arr + a_pos + a_neg + a_off + a_cnt + a_start + a_tick + a_con;
    PT_HIP(hipDeviceSynchronize());   // queued work may still use the old carving
    t->drop_graphs();
    if (need > t->csr_cap) {
        if (t->csr_block) (void)hipFree(t->csr_block);
        t->csr_block = nullptr;
        t->csr_cap = 0;
        PT_HIP(hipMalloc(&t->csr_block, need));
        t->csr_cap = need;
    }
    PT_HIP(hipMemset(t->csr_block, 0, need));   // bucket counts start at zero; the scan re-zeroes them
    char *b = (char *)t->csr_block;
    // the per-chunk memset's block (row uses) first, at the allocation's start
    t->csr.uses = sa ? (int32_t *)b : nullptr; b += a_use;
    t->csr.use_stride = us;
    t->csr.rel_base = E;
    t->csr.lpart = sa ? (float *)b : nullptr; b += a_lp;
    t->fr.gent = sa ? (float *)b : nullptr; b += a_gent;
    t->fr.grel = sa ? (float *)b : nullptr; b += a_grel;
    t->fr.arrive = sa ? (uint64_t *)b : nullptr; b += a_arr;
    t->fr.dp = (int32_t)dp;
    t->csr.pos = (int4 *)b; b += a_pos;
    t->csr.neg = (int32_t *)b; b += a_neg;
    t->csr.off = (int32_t *)b; b += a_off;
    t->csr.cnt = (int32_t *)b; b += a_cnt;
    t->csr.start = (int32_t *)b; b += a_start;
    t->csr.tick = (int32_t *)b; b += a_tick;
    t->csr.contrib = (float *)b;
    t->csr.slot_scale = scm ? 1 : 0;
    t->csr.srec = scm ? (int2 *)b : nullptr;
    t->csr.bases = scm ? (float *)(b + a_srec) : nullptr;
    t->csr.cnt_stride = cs;
    t->csr.start_stride = ss;
    t->csr_bs = bs;
    t->csr_neg = neg;
    t->csr_chunk = chunk;
    // sampling + counting sort in LDS (one workgroup per call, or split over parts) when the plans fit
    // (sets the kernels' LDS attributes here, outside any stream capture)
    t->csr_fused = pt::sample_sort_prepare(bs, neg, E, ss);
    t->csr_part = pt::sample_part_prepare(bs, neg, E, std::min<int64_t>(bs, kPartTarget));
    if (const char *dd = pt_tuning_env("PT_PART_DBG")) t->csr.dbg = atoi(dd);
    // PT_PART_PROF=1: phase timestamps of the split sampler (reported by pt_trainer_run_timed)
    if (const char *pp = pt_tuning_env("PT_PART_PROF")) {
        if (atoi(pp) != 0 && !t->csr.prof) {
            t->prof_cap = kCsrChunk * 1024;   // (call, part) records
            PT_HIP(hipMalloc(&t->csr.prof, sizeof(uint64_t) * 8 * (size_t)t->prof_cap));
        }
    }
    return PT_OK;
}

// Launch recorder for the measurement hook: an event pair around every launch, by kernel kind
// (0 sampling, 1 bucket scan, 2 forward/backward, 3 optimizer apply).
struct Timing {
    // events created up front (hipEventCreate between launches would stall the enqueue and let the
    // GPU idle inside a measured interval)
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    std::vector<std::tuple<int, hipEvent_t, hipEvent_t>> ev;
    int reserve(size_t n) {
        pool.resize(n);
        for (auto &e : pool) PT_HIP(hipEventCreate(&e));
        return PT_OK;
    }
    int begin(int kind, hipStream_t st, hipEvent_t *a) {
        if (used >= pool.size()) return pt::fail(PT_EHIP, "timing event pool exhausted");
        *a = pool[used++];
        PT_HIP(hipEventRecord(*a, st));
        ev.emplace_back(kind, *a, nullptr);
        return PT_OK;
    }
    int end(hipStream_t st) {
        if (used >= pool.size()) return pt::fail(PT_EHIP, "timing event pool exhausted");
        hipEvent_t b = pool[used++];
        PT_HIP(hipEventRecord(b, st));
        std::get<2>(ev.back()) = b;
        return PT_OK;
    }
    ~Timing() {
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

#define PT_TIMED(kind, call)                                  \
    do {                                                      \
        hipEvent_t a_;                                        \
        if (tm && tm->begin(kind, st, &a_)) return PT_EHIP;   \
        PT_HIP(call);                                         \
        if (tm && tm->end(st)) return PT_EHIP;                \
    } while (0)

// Sample `calls` consecutive steps into the counting-sort workspace (pos / neg / destination / start,
// calls <= csr_chunk): sampling + counting sort in LDS, one workgroup per call (then the stream advance)
// or split over parts per call (then the destination resolve + stream advance), or the two-pass form
// (global-atomic counts, separate scan) when no LDS plan fits. `forced` = PT_PATH_* or -1 (automatic).
static int enqueue_sample_chunk(pt_trainer *t, pt_sampler *s, pt::CsrWork &w, int64_t bs, int64_t neg,
                                int64_t bern, int64_t filter, int64_t calls, int forced, hipStream_t st, Timing *tm) {
    const pt::DeviceGraph dg = s->g->dev;
    const int64_t dpp = 1 + 2 * neg;
    const int path = choose_path(t, calls, bs, neg, forced);
    t->last_path = path;
    if (w.uses) PT_HIP(hipMemsetAsync(w.uses, 0, 4 * (size_t)(w.use_stride * calls), st));   // counted by the sampler
    w.rank_only = path == PT_PATH_PART;   // the split sampler leaves bucket ranks (the step resolves them)
    if (path == PT_PATH_FUSED) {
        PT_TIMED(0, pt::launch_sample_sort(dg, s->d_states, s->threads, bs, neg, (int)bern, (int)filter, calls,
                                           t->P.ent_total, w, st));
        PT_TIMED(1, pt::launch_advance(s->d_states, s->threads, bs, dpp * calls, st));
    } else if (path == PT_PATH_PART) {
        const int64_t parts = part_count(t, calls, bs);
        pt::CsrWork wp = w;
        if (wp.prof && calls * parts > t->prof_cap) wp.prof = nullptr;   // record only what the buffer holds
        if (wp.prof) {
            t->prof_calls = calls;
            t->prof_parts = parts;
        }
        PT_TIMED(0, pt::launch_sample_part(dg, s->d_states, s->threads, bs, neg, (int)bern, (int)filter, calls,
                                           parts, t->P.ent_total, wp, st));
    } else {
        PT_TIMED(0, pt::launch_sample_csr(dg, s->d_states, s->threads, bs, neg, (int)bern, (int)filter, calls, w, st));
        PT_TIMED(1, pt::launch_scan_counts(w, t->P.ent_total, calls, s->d_states, s->threads, bs, dpp, st));
    }
    return PT_OK;
}

// Steps of a split-sampler chunk sampled ahead of the first step (0: the chunk is sampled by one launch). The
// batch stream does not depend on the tables, so the chunk's other steps can be sampled by a second launch on
// the trainer's side stream while the first steps train: the chunk's first step then waits for `head` steps'
// sampling instead of the whole chunk's (the driver's 20-step chunk: 52 us). Opt-in (pt_trainer_set_sample_split;
// the tuning build's PT_SAMPLE_SPLIT): measured slower on the driver's command, 38.4 -> 39.6 us per step at
// head 1, 2 or 4 - the side launch's workgroups take the CUs of the steps it runs beside (step 0: 22 -> 43 us)
// and the join across hardware queues leaves the main queue idle for ~11 us (profiles/r05_c2_split_sampling.json).
// Not under the measurement hook (its events time each launch alone) nor for the fused step + apply.
static int64_t sample_split_head(const pt_trainer *t, int path, int64_t calls, const Timing *tm) {
    if (path != PT_PATH_PART || tm) return 0;
    int64_t h = t->split_override;
    if (h < 0) {
        h = 0;
        if (const char *v = pt_tuning_env("PT_SAMPLE_SPLIT")) h = atoll(v);
    }
    return h > 0 && h < calls ? h : 0;
}

// A split-sampler chunk in two launches: the first `head` calls on `st`, the rest on the trainer's side stream
// forked from `st` after it (neither launch advances the streams: join_sample_split does, after both).
static int enqueue_sample_split(pt_trainer *t, pt_sampler *s, pt::CsrWork &w, int64_t bs, int64_t neg, int64_t bern,
                                int64_t filter, int64_t calls, int64_t head, hipStream_t st) {
    const pt::DeviceGraph dg = s->g->dev;
    t->last_path = PT_PATH_PART;
    w.rank_only = 1;
    const int64_t parts = part_count(t, calls, bs);
    pt::CsrWork w0 = w, w1 = pt::csr_view(w, head, bs, neg);
    w0.prof = w1.prof = nullptr;
    w1.tick = w.tick + head;
    PT_HIP(pt::launch_sample_part(dg, s->d_states, s->threads, bs, neg, (int)bern, (int)filter, head, parts,
                                  t->P.ent_total, w0, st, 0, 0));
    PT_HIP(hipEventRecord(t->ev_fork, st));
    PT_HIP(hipStreamWaitEvent(t->side, t->ev_fork, 0));
    PT_HIP(pt::launch_sample_part(dg, s->d_states, s->threads, bs, neg, (int)bern, (int)filter, calls - head, parts,
                                  t->P.ent_total, w1, t->side, head, 0));
    PT_HIP(hipEventRecord(t->ev_join, t->side));
    return PT_OK;
}
// `st` waits for the side launch of enqueue_sample_split, then the streams advance past the chunk's draws
static int join_sample_split(pt_trainer *t, pt_sampler *s, int64_t bs, int64_t neg, int64_t calls, hipStream_t st) {
    PT_HIP(hipStreamWaitEvent(st, t->ev_join, 0));
    PT_HIP(pt::launch_advance(s->d_states, s->threads, bs, (1 + 2 * neg) * calls, st));
    return PT_OK;
}

// whether in-kernel-sampled steps of P take the fused step + apply (carved for in ensure_csr)
static bool step_apply_on(const pt_trainer *t, const pt::StepParams &P) {
    return step_apply_wanted(t) && t->fr.gent && t->csr.uses && pt::step_apply_supported(P, P.batch_size, P.neg);
}

// Enqueue `steps` in-kernel-sampled steps; step i adds its loss to d_losses[i]. Large neg takes the
// counting-sort path: one sampling + one scan launch per chunk of up to kCsrChunk steps (the batch
// stream does not depend on the tables, so it is drawn ahead), then k_step + k_apply per step.
static int enqueue_run(pt_trainer *t, pt_sampler *s, int64_t bs, int64_t neg, int64_t bern, int64_t filter,
                       int64_t steps, float *d_losses, hipStream_t st, Timing *tm = nullptr, bool assign = false) {
    pt::StepParams P = t->P;
    P.loss_assign = assign ? 1 : 0;   // d_losses[i] = step i's loss (no zeroing pass needed)
    P.batch_size = bs;
    P.neg = neg;
    P.inv_count = 1.0f / (float)(bs * neg);
    const int64_t dpp = 1 + 2 * neg;
    const pt::DeviceGraph dg = s->g->dev;
    if (use_csr(neg)) {
        PT_CHECK(t->csr_block, PT_ESTATE, "counting-sort workspace not allocated");
        const int64_t chunk = t->csr_chunk;
        const bool sa = step_apply_on(t, P);
        t->last_step_apply = sa;
        pt::CsrWork w = t->csr;
        if (!sa) w.uses = nullptr;   // (the sampler counts row uses only for the fused kernel)
        for (int64_t c0 = 0; c0 < steps; c0 += chunk) {
            const int64_t calls = std::min(chunk, steps - c0);
            const int path = choose_path(t, calls, bs, neg, sample_mode(t));
            const int64_t head = sa ? 0 : sample_split_head(t, path, calls, tm);
            if (head) {
                int rc = enqueue_sample_split(t, s, w, bs, neg, bern, filter, calls, head, st);
                if (rc) return rc;
            } else {
                int rc = enqueue_sample_chunk(t, s, w, bs, neg, bern, filter, calls, sample_mode(t), st, tm);
                if (rc) return rc;
            }
            t->csr.rank_only = w.rank_only;   // (read by pt_trainer_run_timed's re-timing of the last batch)
            if (sa) {   // one launch per step, then the chunk's losses
                // arrival words back to zero every chunk (the last arriver of a row also clears its word): a step
                // whose arrivals ever miss a row (an aborted launch) cannot carry over past its chunk
                PT_HIP(hipMemsetAsync(t->fr.arrive, 0, 8 * (size_t)(t->P.ent_total + t->P.rel_total), st));
                for (int64_t j = 0; j < calls; ++j)
                    PT_TIMED(2, pt::launch_step_apply(P, pt::csr_view(w, j, bs, neg), t->fr, st));
                if (d_losses)
                    PT_TIMED(3, pt::launch_loss_calls(w.lpart, bs, calls, P.inv_count, P.margin, d_losses + c0,
                                                      P.loss_assign, st));
                continue;
            }
            for (int64_t j = 0; j < calls; ++j) {
                if (head && j == head) {   // the rest of the chunk sampled: join, then advance the streams
                    int rc = join_sample_split(t, s, bs, neg, calls, st);
                    if (rc) return rc;
                }
                const pt::CsrWork v = pt::csr_view(t->csr, j, bs, neg);
                float *loss = d_losses ? d_losses + c0 + j : nullptr;
                PT_TIMED(2, pt::launch_step(P, dg, s->d_states, s->threads, (int)bern, (int)filter, nullptr, nullptr,
                                            nullptr, t->W, loss, st, &v));
                PT_TIMED(3, pt::launch_apply(P, t->W, nullptr, 0, bs, dpp, loss, st, &v));
            }
        }
    } else {
        t->last_path = PT_PATH_SAMPLED;
        t->last_step_apply = false;
        for (int64_t i = 0; i < steps; ++i) {
            float *loss = d_losses ? d_losses + i : nullptr;
            PT_TIMED(2, pt::launch_step(P, dg, s->d_states, s->threads, (int)bern, (int)filter, nullptr, nullptr,
                                        nullptr, t->W, loss, st));
            PT_TIMED(3, pt::launch_apply(P, t->W, s->d_states, s->threads, bs, dpp, loss, st));
        }
    }
    return PT_OK;
}

static int enqueue_external(pt_trainer *t, int64_t bs, int64_t neg, const int64_t *bh, const int64_t *bt,
                            const int64_t *br, float *d_loss, hipStream_t st) {
    pt::StepParams P = t->P;
    P.batch_size = bs;
    P.neg = neg;
    P.inv_count = 1.0f / (float)(bs * neg);
    PT_HIP(pt::launch_step(P, pt::DeviceGraph{}, nullptr, 0, 0, 0, bh, bt, br, t->W, d_loss, st));
    PT_HIP(pt::launch_apply(P, t->W, nullptr, 0, bs, 1 + 2 * neg, d_loss, st));
    return PT_OK;
}

// per-positive loss partials for batches of up to `bs` positives (grown on demand, never during a
// capture: callers prepare before enqueueing)
static int ensure_lpart(pt_trainer *t, int64_t bs) {
    if (bs <= t->lpart_cap) return PT_OK;
    PT_HIP(hipDeviceSynchronize());   // queued work may still use the old buffer
    t->drop_graphs();
    if (t->W.lpart) (void)hipFree(t->W.lpart);
    t->W.lpart = nullptr;
    t->lpart_cap = 0;
    PT_HIP(hipMalloc(&t->W.lpart, sizeof(float) * (size_t)bs));
    t->lpart_cap = bs;
    return PT_OK;
}

static int prepare_sampled(pt_trainer *t, pt_sampler *s, int64_t bs, int64_t neg, int64_t steps) {
    int rc = check_step_args(t->P, s, bs, neg, nullptr);
    if (rc) return rc;
    rc = ensure_lpart(t, bs);
    if (rc) return rc;
    rc = s->g->upload();
    if (rc) return rc;
    (void)steps;
    if (use_csr(neg)) return ensure_csr(t, bs, neg);
    return PT_OK;
}

// ---- reference-order mode (ordered.hip): workspace for batches of up to `seq` slots
static int ensure_ordered(pt_trainer *t, int64_t seq) {
    const int64_t D = t->P.dim;
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t need = 3 * al(8 * seq) + 3 * al(4 * seq) + al(16 * (size_t)seq * D);
    if (need <= t->ord_cap) return PT_OK;
    PT_HIP(hipDeviceSynchronize());   // queued ordered steps may still use the old block
    if (t->ord_block) (void)hipFree(t->ord_block);
    t->ord_block = nullptr;
    t->ord_cap = 0;
    PT_HIP(hipMalloc(&t->ord_block, need));
    t->ord_cap = need;
    char *b = (char *)t->ord_block;
    t->ord_h = (int64_t *)b; b += al(8 * seq);
    t->ord_t = (int64_t *)b; b += al(8 * seq);
    t->ord_r = (int64_t *)b; b += al(8 * seq);
    t->ord_y = (float *)b; b += al(4 * seq);
    t->ord_score = (float *)b; b += al(4 * seq);
    t->ord_ds = (float *)b; b += al(4 * seq);
    t->ord_g = (float *)b;
    return PT_OK;
}

static int enqueue_ordered(pt_trainer *t, int64_t bs, int64_t neg, const int64_t *bh, const int64_t *bt,
                           const int64_t *br, float *loss, int assign, hipStream_t st) {
    const pt::StepParams &P = t->P;
    pt::OrderedStep S{};
    S.model = P.model; S.p_norm = P.p_norm; S.norm_flag = P.norm_flag; S.opt = P.opt;
    S.lr = P.lr; S.margin = P.margin;
    S.ent_total = P.ent_total; S.rel_total = P.rel_total; S.dim = P.dim;
    S.ent = P.ent; S.rel = P.rel; S.normv = P.normv;
    S.ent_acc = P.ent_acc; S.rel_acc = P.rel_acc; S.norm_acc = P.norm_acc;
    S.h = bh; S.t = bt; S.r = br;
    S.bs = bs; S.neg = neg; S.seq = bs * (1 + neg);
    S.score = t->ord_score; S.ds = t->ord_ds;
    S.gh = t->ord_g; S.gt = S.gh + S.seq * P.dim; S.gr = S.gt + S.seq * P.dim; S.gw = S.gr + S.seq * P.dim;
    PT_HIP(pt::launch_ordered_step(S, loss, assign, st));
    return PT_OK;
}

// `steps` sampled steps in reference order: k_sample's batch (bit-identical to sampling()), then the step
static int enqueue_ordered_run(pt_trainer *t, pt_sampler *s, int64_t bs, int64_t neg, int64_t bern, int64_t filter,
                               int64_t steps, float *d_losses, int assign, hipStream_t st) {
    PT_CHECK(s && s->g && s->d_states, PT_ESTATE, "in-kernel sampling needs a sampler bound to a graph");
    PT_CHECK(s->g->ent_total > 1, PT_EINVAL, "graph needs at least two entities");
    PT_CHECK(s->g->ent_total <= t->P.ent_total && s->g->rel_total <= t->P.rel_total, PT_EINVAL,
             "graph ids exceed the model tables");
    int rc = s->g->upload();
    if (rc) return rc;
    rc = ensure_ordered(t, bs * (1 + neg));
    if (rc) return rc;
    t->last_path = -1;
    for (int64_t i = 0; i < steps; ++i) {
        PT_HIP(pt::launch_sample(s->g->dev, s->d_states, s->threads, bs, neg, 0, 0, (int)bern, (int)filter, t->ord_h,
                                 t->ord_t, t->ord_r, t->ord_y, st));
        PT_HIP(pt::launch_advance(s->d_states, s->threads, bs, 1 + 2 * neg, st));
        rc = enqueue_ordered(t, bs, neg, t->ord_h, t->ord_t, t->ord_r, d_losses ? d_losses + i : nullptr, assign, st);
        if (rc) return rc;
    }
    return PT_OK;
}

extern "C" int pt_trainer_set_sampling(pt_trainer *t, int32_t path, int64_t parts) {
    PT_CHECK(t, PT_EINVAL, "null trainer");
    PT_CHECK(path >= -1 && path <= PT_PATH_PART, PT_EINVAL, "sampling path must be -1 or PT_PATH_FUSED/PART/TWO_PASS");
    PT_CHECK(parts >= 0, PT_EINVAL, "parts must be >= 0");
    t->path_override = path;
    t->parts_override = parts;
    t->drop_graphs();   // captured epochs hold the previous choice
    return PT_OK;
}

extern "C" int pt_trainer_set_sample_split(pt_trainer *t, int64_t head) {
    PT_CHECK(t, PT_EINVAL, "null trainer");
    PT_CHECK(head >= -1, PT_EINVAL, "head must be >= -1");
    t->split_override = head;
    t->drop_graphs();   // captured epochs hold the previous choice
    return PT_OK;
}

extern "C" int pt_trainer_set_deterministic(pt_trainer *t, int32_t on) {
    PT_CHECK(t, PT_EINVAL, "null trainer");
    PT_CHECK(!on || pt::ordered_dim_supported(t->P.dim), PT_ENOTSUP, "reference-order mode: dim too large");
    t->ordered = on != 0;
    return PT_OK;
}
extern "C" int pt_trainer_get_deterministic(const pt_trainer *t) { return t && t->ordered ? 1 : 0; }

extern "C" int pt_trainer_step(pt_trainer *t, pt_sampler *s, int64_t bs, int64_t neg, int64_t bern, int64_t filter,
                               const int64_t *d_bh, const int64_t *d_bt, const int64_t *d_br, float *d_loss,
                               void *stream) {
    PT_CHECK(t, PT_EINVAL, "null trainer");
    if (d_bh) {
        PT_CHECK(d_bt && d_br, PT_EINVAL, "external batch needs h, t and r arrays");
        PT_CHECK(bs > 0 && neg > 0, PT_EINVAL, "batch_size and neg_ent must be positive");
        if (t->ordered) {
            int rc = ensure_ordered(t, bs * (1 + neg));
            if (rc) return rc;
            return enqueue_ordered(t, bs, neg, d_bh, d_bt, d_br, d_loss, 0, (hipStream_t)stream);
        }
        int rc = ensure_lpart(t, bs);
        if (rc) return rc;
        return enqueue_external(t, bs, neg, d_bh, d_bt, d_br, d_loss, (hipStream_t)stream);
    }
    PT_CHECK(bs > 0 && neg > 0, PT_EINVAL, "batch_size and neg_ent must be positive");
    if (t->ordered) return enqueue_ordered_run(t, s, bs, neg, bern, filter, 1, d_loss, 0, (hipStream_t)stream);
    int rc = prepare_sampled(t, s, bs, neg, 1);
    if (rc) return rc;
    return enqueue_run(t, s, bs, neg, bern, filter, 1, d_loss, (hipStream_t)stream);
}

// `steps` in-kernel-sampled steps launched one by one with an event pair around every launch on
// `stream` (measurement hook for bench.py's roofline). ms4[k] = total duration of kernel kind k
// (0 sampling, 1 bucket scan, 2 forward/backward, 3 optimizer) divided by `steps`. Synchronizes.
extern "C" int pt_trainer_run_timed(pt_trainer *t, pt_sampler *s, int64_t bs, int64_t neg, int64_t bern,
                                    int64_t filter, int64_t steps, float *d_losses, float *ms4, void *stream) {
    PT_CHECK(t && ms4 && steps > 0, PT_EINVAL, "pt_trainer_run_timed: bad argument");
    PT_CHECK(!t->ordered, PT_ENOTSUP, "pt_trainer_run_timed times the fast path (reference-order mode is on)");
    int rc = prepare_sampled(t, s, bs, neg, steps);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    Timing tm;
    rc = tm.reserve((size_t)(8 * steps + 64));
    if (rc) return rc;
    // hold the stream in a short spin kernel while the host enqueues every measured launch, so each
    // kernel starts as soon as its predecessor ends (no host-side gaps inside an event pair)
    PT_HIP(pt::launch_spin(20000, st));
    rc = enqueue_run(t, s, bs, neg, bern, filter, steps, d_losses, st, &tm, true);
    if (rc) return rc;
    PT_HIP(hipStreamSynchronize(st));
    double tot[4] = {0, 0, 0, 0};
    for (auto &e : tm.ev) {
        float ms = 0;
        PT_HIP(hipEventElapsedTime(&ms, std::get<1>(e), std::get<2>(e)));
        tot[std::get<0>(e)] += ms;
    }
    for (int k = 0; k < 4; ++k) ms4[k] = (float)(tot[k] / (double)steps);
    if (t->csr.prof && t->last_path == PT_PATH_PART && t->prof_calls > 0) {   // split sampler phases of the last chunk
        const int64_t calls = t->prof_calls, parts = t->prof_parts;
        std::vector<uint64_t> pr((size_t)(8 * calls * parts));
        PT_HIP(hipMemcpy(pr.data(), t->csr.prof, 8 * pr.size(), hipMemcpyDeviceToHost));
        uint64_t t0 = ~0ull, tend = 0;
        double ph[7] = {0}, mx[7] = {0};
        int64_t n_last = 0;
        double last5 = 0, last6 = 0;
        for (int64_t i = 0; i < calls * parts; ++i) t0 = std::min(t0, pr[8 * i]);
        for (int64_t i = 0; i < calls * parts; ++i) {
            const uint64_t *q = &pr[8 * i];
            for (int k = 1; k <= 4; ++k) {
                ph[k] += (double)(q[k] - q[k - 1]);
                mx[k] = std::max(mx[k], (double)(q[k] - t0));
            }
            mx[0] = std::max(mx[0], (double)(q[0] - t0));
            if (q[7]) {
                ++n_last;
                last5 += (double)(q[5] - q[4]);
                last6 += (double)(q[6] - q[5]);
                tend = std::max(tend, q[6]);
            }
        }
        const double n = (double)(calls * parts);
        fprintf(stderr,
                "part-prof calls %ld parts %ld: avg us positives %.2f slots %.2f reserve %.2f rank+ticket %.2f | "
                "last exchange %.2f scan %.2f | latest start %.2f, phase ends (max from first start) %.2f %.2f %.2f "
                "%.2f, kernel end %.2f\n",
                (long)calls, (long)parts, ph[1] / n / 100, ph[2] / n / 100, ph[3] / n / 100, ph[4] / n / 100,
                last5 / std::max<int64_t>(n_last, 1) / 100, last6 / std::max<int64_t>(n_last, 1) / 100, mx[0] / 100,
                mx[1] / 100, mx[2] / 100, mx[3] / 100, mx[4] / 100, (double)(tend - t0) / 100);
    }
    if (!use_csr(neg)) return PT_OK;
    // Counting-sort path: the per-step kernels are re-timed back to back (as a captured epoch runs
    // them), one event pair per loop instead of one per launch, on the last pre-sampled batch:
    //   loop 1: `steps` x (forward/backward, apply)  -> T_sa;   loop 2: `steps` x forward/backward -> T_s
    // ms4[2] = T_s / steps, ms4[3] = (T_sa - T_s) / steps. The tables, Adagrad state, gradient rows and
    // flags are restored afterwards, so training state is exactly as the measured run left it.
    pt::StepParams P = t->P;
    P.batch_size = bs;
    P.neg = neg;
    P.inv_count = 1.0f / (float)(bs * neg);
    const int64_t E = P.ent_total, R = P.rel_total, D = P.dim, dpp = 1 + 2 * neg;
    std::vector<std::pair<float *, size_t>> keep = {{P.ent, 4 * E * D}, {P.rel, 4 * R * D}};
    if (P.normv) keep.push_back({P.normv, 4 * R * D});
    if (P.opt != 0) {
        keep.push_back({P.ent_acc, 4 * E * D});
        keep.push_back({P.rel_acc, 4 * R * D});
        if (P.norm_acc) keep.push_back({P.norm_acc, 4 * R * D});
    }
    size_t nb = 0;
    for (auto &k : keep) nb += k.second;
    char *bak = nullptr;
    PT_HIP(hipMalloc(&bak, nb));
    size_t off = 0;
    for (auto &k : keep) {
        PT_HIP(hipMemcpyAsync(bak + off, k.first, k.second, hipMemcpyDeviceToDevice, st));
        off += k.second;
    }
    const pt::DeviceGraph dg = s->g->dev;
    const pt::CsrWork v = pt::csr_view(t->csr, 0, bs, neg);
    hipEvent_t ev[4] = {tm.pool[0], tm.pool[1], tm.pool[2], tm.pool[3]};
    int erc = PT_OK;
    if (pt::launch_spin(20000, st) != hipSuccess || hipEventRecord(ev[0], st) != hipSuccess) erc = PT_EHIP;
    // the fused step + apply: loop 1 only (ms4[3] keeps the chunks' loss kernels from the pass above)
    const bool sa = t->last_step_apply;
    for (int64_t i = 0; i < steps && !erc; ++i) {
        if (sa) {
            if (pt::launch_step_apply(P, v, t->fr, st) != hipSuccess) erc = PT_EHIP;
            continue;
        }
        if (pt::launch_step(P, dg, s->d_states, s->threads, (int)bern, (int)filter, nullptr, nullptr, nullptr, t->W,
                            nullptr, st, &v) != hipSuccess ||
            pt::launch_apply(P, t->W, nullptr, 0, bs, dpp, nullptr, st, &v) != hipSuccess)
            erc = PT_EHIP;
    }
    if (!erc && (hipEventRecord(ev[1], st) != hipSuccess || pt::launch_spin(20000, st) != hipSuccess ||
                 hipEventRecord(ev[2], st) != hipSuccess))
        erc = PT_EHIP;
    for (int64_t i = 0; i < steps && !erc && !sa; ++i) {
        if (pt::launch_step(P, dg, s->d_states, s->threads, (int)bern, (int)filter, nullptr, nullptr, nullptr, t->W,
                            nullptr, st, &v) != hipSuccess)
            erc = PT_EHIP;
    }
    if (!erc && hipEventRecord(ev[3], st) != hipSuccess) erc = PT_EHIP;
    // restore
    off = 0;
    for (auto &k : keep) {
        if (hipMemcpyAsync(k.first, bak + off, k.second, hipMemcpyDeviceToDevice, st) != hipSuccess) erc = PT_EHIP;
        off += k.second;
    }
    if (hipMemsetAsync(t->ws_block, 0, t->ws_bytes, st) != hipSuccess) erc = PT_EHIP;
    const hipError_t se = hipStreamSynchronize(st);
    (void)hipFree(bak);
    if (erc) return pt::fail(erc, "pt_trainer_run_timed: isolation timing launch failed");
    PT_HIP(se);
    float t_sa = 0, t_s = 0;
    PT_HIP(hipEventElapsedTime(&t_sa, ev[0], ev[1]));
    PT_HIP(hipEventElapsedTime(&t_s, ev[2], ev[3]));
    if (sa) {
        ms4[2] = t_sa / (float)steps;
    } else {
        ms4[2] = t_s / (float)steps;
        ms4[3] = (t_sa - t_s) / (float)steps;
    }
    return PT_OK;
}

extern "C" int pt_trainer_set_step_apply(pt_trainer *t, int32_t on) {
    PT_CHECK(t, PT_EINVAL, "null trainer");
    if (t->step_apply_on != (on != 0)) t->csr_bs = 0;   // re-carve the workspace: the fused kernel's state only when on
    t->step_apply_on = on != 0;
    t->drop_graphs();   // captured epochs hold the previous choice
    return PT_OK;
}
extern "C" int pt_trainer_step_apply(const pt_trainer *t) { return t && t->last_step_apply ? 1 : 0; }

extern "C" int pt_trainer_set_slot_scale(pt_trainer *t, int32_t on) {
    PT_CHECK(t, PT_EINVAL, "null trainer");
    if (t->slot_scale_on != (on != 0)) t->csr_bs = 0;   // re-carve the workspace (slot records / base rows)
    t->slot_scale_on = on != 0;
    t->drop_graphs();
    return PT_OK;
}
extern "C" int pt_trainer_slot_scale(const pt_trainer *t) { return t && t->csr.slot_scale ? 1 : 0; }

extern "C" int pt_trainer_last_path(const pt_trainer *t) { return t ? t->last_path : -1; }

extern "C" int pt_trainer_sample_csr(pt_trainer *t, pt_sampler *s, int64_t bs, int64_t neg, int64_t bern,
                                     int64_t filter, int64_t calls, int32_t path, int32_t *h_pos, int32_t *h_neg,
                                     int32_t *h_dst, int32_t *h_start, void *stream) {
    PT_CHECK(t && s && h_pos && h_neg && h_dst && h_start, PT_EINVAL, "pt_trainer_sample_csr: null argument");
    PT_CHECK(calls > 0, PT_EINVAL, "pt_trainer_sample_csr: calls must be positive");
    PT_CHECK(path >= -1 && path <= PT_PATH_PART, PT_EINVAL, "pt_trainer_sample_csr: path must be -1 or PT_PATH_*");
    int rc = prepare_sampled(t, s, bs, neg, calls);
    if (rc) return rc;
    if (!t->csr_block) {   // small neg runs the in-step sampler; carve the counting-sort workspace anyway
        rc = ensure_csr(t, bs, neg);
        if (rc) return rc;
    }
    PT_CHECK(calls <= t->csr_chunk, PT_EINVAL, "pt_trainer_sample_csr: calls exceeds the workspace chunk");
    if (path == PT_PATH_FUSED) PT_CHECK(t->csr_fused, PT_ENOTSUP, "fused sampling plan does not fit LDS");
    if (path == PT_PATH_PART)
        PT_CHECK(t->csr_part && pt::sample_part_fits(bs, neg, t->P.ent_total, part_count(t, calls, bs)), PT_ENOTSUP,
                 "split sampling plan does not fit LDS");
    hipStream_t st = (hipStream_t)stream;
    const int64_t head = path == PT_PATH_PART && t->split_override > 0 && t->split_override < calls ? t->split_override
                                                                                                    : 0;
    if (head) {   // the split pair (pt_trainer_set_sample_split), joined before the copies
        rc = enqueue_sample_split(t, s, t->csr, bs, neg, bern, filter, calls, head, st);
        if (!rc) rc = join_sample_split(t, s, bs, neg, calls, st);
    } else {
        rc = enqueue_sample_chunk(t, s, t->csr, bs, neg, bern, filter, calls, path, st, nullptr);
    }
    if (rc) return rc;
    const pt::CsrWork &w = t->csr;
    const int64_t E = t->P.ent_total, slots = bs * neg;
    std::vector<int4> pos((size_t)(calls * bs));
    PT_HIP(hipMemcpyAsync(pos.data(), w.pos, sizeof(int4) * pos.size(), hipMemcpyDeviceToHost, st));
    PT_HIP(hipMemcpyAsync(h_neg, w.neg, 4 * (size_t)(calls * slots), hipMemcpyDeviceToHost, st));
    PT_HIP(hipMemcpyAsync(h_dst, w.off, 4 * (size_t)(calls * slots), hipMemcpyDeviceToHost, st));
    PT_HIP(hipMemcpy2DAsync(h_start, 4 * (size_t)(E + 1), w.start, 4 * (size_t)w.start_stride, 4 * (size_t)(E + 1),
                            (size_t)calls, hipMemcpyDeviceToHost, st));
    PT_HIP(hipStreamSynchronize(st));
    if (w.rank_only)   // split sampler: ranks inside the buckets -> destination rows
        for (int64_t c = 0; c < calls; ++c)
            for (int64_t o = 0; o < slots; ++o)
                h_dst[c * slots + o] += h_start[c * (E + 1) + (h_neg[c * slots + o] >> 1)];
    for (size_t i = 0; i < pos.size(); ++i) {
        h_pos[3 * i] = pos[i].x;
        h_pos[3 * i + 1] = pos[i].y;
        h_pos[3 * i + 2] = pos[i].z;
    }
    return PT_OK;
}

extern "C" int pt_trainer_run(pt_trainer *t, pt_sampler *s, int64_t bs, int64_t neg, int64_t bern, int64_t filter,
                              int64_t steps, float *d_losses, void *stream) {
    PT_CHECK(t && d_losses, PT_EINVAL, "pt_trainer_run: null argument");
    PT_CHECK(steps > 0, PT_EINVAL, "steps must be positive");
    if (t->ordered) {
        PT_CHECK(bs > 0 && neg > 0, PT_EINVAL, "batch_size and neg_ent must be positive");
        return enqueue_ordered_run(t, s, bs, neg, bern, filter, steps, d_losses, 1, (hipStream_t)stream);
    }
    int rc = prepare_sampled(t, s, bs, neg, steps);
    if (rc) return rc;
    GraphKey key{s, s->g->dev.rec, d_losses, s->d_states, bs, neg, bern, filter, steps};
    auto it = t->graphs.find(key);
    if (it == t->graphs.end()) {
        hipGraph_t graph;
        PT_HIP(hipStreamBeginCapture(t->cap, hipStreamCaptureModeThreadLocal));
        int erc = PT_OK;
        erc = enqueue_run(t, s, bs, neg, bern, filter, steps, d_losses, t->cap, nullptr, true);
        hipError_t ce = hipStreamEndCapture(t->cap, &graph);
        if (erc) return erc;
        PT_HIP(ce);
        hipGraphExec_t exec;
        hipError_t ie = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        PT_HIP(ie);
        it = t->graphs.emplace(key, exec).first;
    }
    PT_HIP(hipGraphLaunch(it->second, (hipStream_t)stream));
    return PT_OK;
}

extern "C" int pt_score(const pt_model_desc *m, int32_t mode, const int64_t *d_h, const int64_t *d_t,
                        const int64_t *d_r, int64_t n, float *d_out, void *stream) {
    pt::StepParams P{};
    pt_model_desc mm = *m;
    if (!mm.ent_acc) { mm.opt = PT_SGD; }
    int rc = desc_to_params(&mm, P);
    if (rc) return rc;
    PT_CHECK(mode >= 0 && mode <= 2, PT_EINVAL, "mode must be 0 (normal), 1 (head_batch) or 2 (tail_batch)");
    PT_CHECK(d_h && d_t && d_r && d_out, PT_EINVAL, "pt_score: null argument");
    PT_HIP(pt::launch_score(P, mode, d_h, d_t, d_r, n, d_out, (hipStream_t)stream));
    return PT_OK;
}

extern "C" int pt_score_queries(const pt_model_desc *m, int32_t side, const int64_t *d_qh, const int64_t *d_qt,
                                const int64_t *d_qr, int64_t nq, float *d_out, void *stream) {
    pt::StepParams P{};
    pt_model_desc mm = *m;
    if (!mm.ent_acc) mm.opt = PT_SGD;
    int rc = desc_to_params(&mm, P);
    if (rc) return rc;
    PT_CHECK(side == 0 || side == 1, PT_EINVAL, "side must be 0 (head prediction) or 1 (tail prediction)");
    PT_CHECK(nq <= 65535, PT_EINVAL, "at most 65535 queries per call");
    PT_CHECK((d_qh && d_qt && d_qr && d_out) || nq == 0, PT_EINVAL, "pt_score_queries: null argument");
    PT_HIP(pt::launch_score_queries(P, side, d_qh, d_qt, d_qr, nq, P.ent_total, d_out, (hipStream_t)stream));
    return PT_OK;
}

extern "C" int pt_score_rows(const pt_model_desc *m, int32_t side, const int64_t *d_qh, const int64_t *d_qt,
                             const int64_t *d_qr, int64_t nq, float *d_out, void *stream) {
    pt::StepParams P{};
    pt_model_desc mm = *m;
    if (!mm.ent_acc) mm.opt = PT_SGD;
    int rc = desc_to_params(&mm, P);
    if (rc) return rc;
    PT_CHECK(side == 0 || side == 1, PT_EINVAL, "side must be 0 (head prediction) or 1 (tail prediction)");
    PT_CHECK(nq <= 65535, PT_EINVAL, "at most 65535 queries per call");
    PT_CHECK((d_qh && d_qt && d_qr && d_out) || nq == 0, PT_EINVAL, "pt_score_rows: null argument");
    PT_HIP(pt::launch_score_queries(P, side, d_qh, d_qt, d_qr, nq, P.ent_total, d_out, (hipStream_t)stream, 1));
    return PT_OK;
}

// Test.h:213-223 + :398-454 accumulation for n ranked queries (float accumulators, same order)
extern "C" int pt_lp_metrics(const int64_t *rank_head, const int64_t *frank_head, const int64_t *rank_tail,
                             const int64_t *frank_tail, int64_t n, float *metrics) {
    PT_CHECK(metrics && (n == 0 || (rank_head && frank_head && rank_tail && frank_tail)), PT_EINVAL,
             "pt_lp_metrics: null argument");
    float lf10 = 0, lf3 = 0, lf1 = 0, lfr = 0, lfi = 0, rf10 = 0, rf3 = 0, rf1 = 0, rfr = 0, rfi = 0;
    float l10 = 0, l3 = 0, l1 = 0, lr = 0, li = 0, r10 = 0, r3 = 0, r1 = 0, rr = 0, ri = 0;
    for (int64_t q = 0; q < n; ++q) {
        const int64_t a = rank_head[q], fa = frank_head[q], b = rank_tail[q], fb = frank_tail[q];
        if (fa < 10) lf10 += 1; if (a < 10) l10 += 1; if (fa < 3) lf3 += 1; if (a < 3) l3 += 1;
        if (fa < 1) lf1 += 1; if (a < 1) l1 += 1;
        lfr += (float)(fa + 1); lr += (float)(1 + a);
        lfi = (float)((double)lfi + 1.0 / (double)(fa + 1)); li = (float)((double)li + 1.0 / (double)(a + 1));
        if (fb < 10) rf10 += 1; if (b < 10) r10 += 1; if (fb < 3) rf3 += 1; if (b < 3) r3 += 1;
        if (fb < 1) rf1 += 1; if (b < 1) r1 += 1;
        rfr += (float)(1 + fb); rr += (float)(1 + b);
        rfi = (float)((double)rfi + 1.0 / (double)(1 + fb)); ri = (float)((double)ri + 1.0 / (double)(1 + b));
    }
    const float N = (float)n;
    lfr /= N; rfr /= N; lfi /= N; rfi /= N; lf10 /= N; lf3 /= N; lf1 /= N; rf10 /= N; rf3 /= N; rf1 /= N;
    lr /= N; rr /= N; li /= N; ri /= N; l10 /= N; l3 /= N; l1 /= N; r10 /= N; r3 /= N; r1 /= N;
    metrics[0] = (lfi + rfi) / 2; metrics[1] = (lfr + rfr) / 2; metrics[2] = (lf10 + rf10) / 2;
    metrics[3] = (lf3 + rf3) / 2; metrics[4] = (lf1 + rf1) / 2;
    metrics[5] = (li + ri) / 2; metrics[6] = (lr + rr) / 2; metrics[7] = (l10 + r10) / 2;
    metrics[8] = (l3 + r3) / 2; metrics[9] = (l1 + r1) / 2;
    return PT_OK;
}

// ======================================================================== universes ==============
extern "C" int pt_universe_build(const pt_graph *g, int64_t seed, int64_t threads, int64_t tc, float balance,
                                 pt_universe **out) {
    PT_CHECK(g && out, PT_EINVAL, "pt_universe_build: null argument");
    PT_CHECK(threads > 0 && threads <= 64 && tc > 0, PT_EINVAL, "bad threads / triple constraint");
    auto *u = new pt_universe();
    pt::GlibcRand rng((uint32_t)seed);   // srand(seed) (Random.h:37-42)
    u->u.seeds.resize((size_t)threads);
    for (auto &x : u->u.seeds) x = (uint64_t)(int64_t)rng.next();   // randReset (Random.h:10-15)
    pt::build_universe(g->g, rng, tc, balance, u->u);
    *out = u;
    return PT_OK;
}

extern "C" int pt_universe_build_many(const pt_graph *g, int64_t n, const int64_t *seeds, int64_t threads,
                                      const int64_t *tcs, const float *balances, int64_t n_workers, pt_universe **out) {
    PT_CHECK(g && seeds && tcs && balances && out, PT_EINVAL, "pt_universe_build_many: null argument");
    if (n_workers <= 0) n_workers = std::max(1u, std::thread::hardware_concurrency());
    n_workers = std::min<int64_t>(n_workers, std::max<int64_t>(n, 1));
    std::atomic<int64_t> next{0};
    std::atomic<int> err{0};
    auto work = [&]() {
        for (int64_t i; (i = next.fetch_add(1)) < n;) {
            pt_universe *u = nullptr;
            int rc = pt_universe_build(g, seeds[i], threads, tcs[i], balances[i], &u);
            if (rc) err = rc;
            out[i] = u;
        }
    };
    std::vector<std::thread> pool;
    for (int64_t w = 1; w < n_workers; ++w) pool.emplace_back(work);
    work();
    for (auto &th : pool) th.join();
    return err.load();
}
extern "C" int pt_universe_free(pt_universe *u) {
    delete u;
    return PT_OK;
}
extern "C" int64_t pt_universe_ent_total(const pt_universe *u) { return u ? u->u.g.ent_total : -1; }
extern "C" int64_t pt_universe_rel_total(const pt_universe *u) { return u ? u->u.g.rel_total : -1; }
extern "C" int64_t pt_universe_train_total(const pt_universe *u) { return u ? u->u.g.train_total : -1; }
extern "C" int pt_universe_remaps(const pt_universe *u, int64_t *ent_remap, int64_t *rel_remap) {
    PT_CHECK(u, PT_EINVAL, "null universe");
    if (ent_remap) std::copy(u->u.ent_remap.begin(), u->u.ent_remap.end(), ent_remap);
    if (rel_remap) std::copy(u->u.rel_remap.begin(), u->u.rel_remap.end(), rel_remap);
    return PT_OK;
}
extern "C" pt_graph *pt_universe_graph(pt_universe *u) {
    // pt_graph is a thin wrapper over pt::Graph; the universe owns it
    return u ? reinterpret_cast<pt_graph *>(&u->u.g) : nullptr;
}
extern "C" int pt_universe_seeds(const pt_universe *u, uint64_t *seeds) {
    PT_CHECK(u && seeds, PT_EINVAL, "null argument");
    std::copy(u->u.seeds.begin(), u->u.seeds.end(), seeds);
    return PT_OK;
}

// Streams of the universe trainer's concurrent class launches: created once per device for the whole process
// and shared by every set. Each is created with a CU mask that covers every CU: the runtime gives such a stream
// a hardware queue of its own instead of sharing one of the process's GPU_MAX_HW_QUEUES (4) queues with the
// caller's streams. With plain streams, a process that already held streams of its own (torch's, the C2 trainer's
// capture stream) got two class launches on one queue, where they ran one after the other (round 4: the C3 set
// 58.7 ms in the default bench process against 35.7 ms standalone).
namespace {
struct ClassStreamPool {
    std::mutex mu;
    std::map<std::pair<int, int>, std::vector<hipStream_t>> by_dev;   // (device, mode) -> streams
    // destroyed when the library is unloaded (process exit): the HIP runtime, loaded before this library, is
    // finalized after it, so the queues are released while it still runs
    ~ClassStreamPool() {
        for (auto &kv : by_dev) {
            if (hipSetDevice(kv.first.first) != hipSuccess) continue;
            for (hipStream_t q : kv.second) (void)hipStreamDestroy(q);
        }
    }
};
ClassStreamPool &class_stream_pool() {
    static ClassStreamPool p;
    return p;
}
// mode 1: full-CU-mask streams (dedicated hardware queues; the product's choice); tuning builds also take
// PT_UNI_STREAMS = 0 (round 4: per-set plain side streams, class 0 on the caller's stream), 2 (highest-priority
// streams: their own queue pool), 3 (plain library streams)
int class_stream_mode() {
    static const int m = [] {
        const char *v = pt_tuning_env("PT_UNI_STREAMS");
        return v ? atoi(v) : 1;
    }();
    return m;
}
hipError_t class_streams(int device, int mode, size_t n, std::vector<hipStream_t> *out) {
    ClassStreamPool &P = class_stream_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    auto &v = P.by_dev[{device, mode}];
    while (v.size() < n) {
        hipStream_t q = nullptr;
        hipError_t e = hipSuccess;
        if (mode == 1) {
            int cus = 0;
            e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
            if (e != hipSuccess) return e;
            std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0u);
            for (int c = 0; c < cus; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
            e = hipExtStreamCreateWithCUMask(&q, (uint32_t)mask.size(), mask.data());
        } else if (mode == 2) {
            int lo = 0, hi = 0;
            e = hipDeviceGetStreamPriorityRange(&lo, &hi);
            if (e == hipSuccess) e = hipStreamCreateWithPriority(&q, hipStreamNonBlocking, hi);
        } else {
            e = hipStreamCreateWithFlags(&q, hipStreamNonBlocking);
        }
        if (e != hipSuccess) return e;
        v.push_back(q);
    }
    out->assign(v.begin(), v.begin() + (std::ptrdiff_t)n);
    return hipSuccess;
}
}  // namespace

// Team universes (universes_team.h): the widest team a set may give one universe (1: none), process-wide like the
// reference's global state; read when a set is created
namespace {
std::atomic<int> g_team_width{1};
}
extern "C" int pt_set_universe_team_width(int32_t w) {
    PT_CHECK(w == 1 || w == 2 || w == 4, PT_EINVAL, "pt_set_universe_team_width: 1, 2 or 4");
    g_team_width.store(w);
    return PT_OK;
}
extern "C" int32_t pt_get_universe_team_width(void) { return g_team_width.load(); }


// Train many universes with the persistent multi-universe kernel (universes.hip).
struct pt_universe_set {
    int32_t model = 0, p_norm = 1, norm_flag = 1, opt = PT_ADAGRAD;
    int64_t bern = 0, filter = 0, neg = 1;
    int device = -1;
    void *arena = nullptr;
    pt::UniverseDev *d_us = nullptr;      // inside the arena, by row shape, longest-first inside a shape
    int *d_counter = nullptr;             // work-queue counters, one per shape group (inside the arena)
    struct Group {
        int shape;
        int64_t off, n;
        double work;
        int64_t share = 1;   // workgroups (= CUs) of its launch
        // team launch (shape class >= kUniTeamBase): [grid][2] universe (index from off) and member (-1: idle)
        int32_t *d_map = nullptr;
        int64_t grid = 0;
    };
    uint32_t *d_team_sync = nullptr;      // team universes' arrival counters (inside the arena, zeroed per call)
    int64_t n_team_sync = 0;
    pt::UniverseLaunch team_cfg;          // the team launches' LDS plan
    pt::TeamDev *d_teams = nullptr;       // [host]: team universes' exchange state (inside the team arena)
    std::vector<int> host_team_w;         // [host]: team width (1: a workgroup of its own)
    std::vector<Group> groups;            // runs of d_us with one shape class (one kernel launch each)
    std::vector<hipStream_t> streams;     // PT_UNI_STREAMS=0 only: per-set side streams (else the process pool's)
    std::vector<hipEvent_t> events;
    std::vector<hipEvent_t> t_start, t_stop;   // per group launch: timing events of the last train call
    bool timed = false;                        // the last train call recorded them
    pt::UniverseLaunch cfg;
    std::vector<pt::UniverseDev> host;    // same order; loss pointers patched per train call
    std::vector<int64_t> host_loss_off;
    std::vector<int64_t> host_of_job;     // job index -> index in host / d_us
    std::vector<uint64_t> seeds0;         // [host][64]: the jobs' LCG states at creation (pt_universe_set_reset)
    void *graph_arena = nullptr;          // the universes' device graphs (one allocation, one copy)
    uint64_t *prof = nullptr;             // PT_UNI_PROF=1: [n][64] cycle counters + shape (+ stamps) (device)
    // reference-order (deterministic) mode (pt_universe_set_deterministic): ordered.hip's universe kernel
    bool ordered = false;
    void *ord_arena = nullptr;            // per universe [4][seq][dim] gradient rows
    int64_t ord_max_seq = 0;
    void *team_arena = nullptr;           // team universes: partials, arrival counters, launch maps
    ~pt_universe_set() {
        if (team_arena) (void)hipFree(team_arena);
        for (auto e : events) (void)hipEventDestroy(e);
        for (auto e : t_start) (void)hipEventDestroy(e);
        for (auto e : t_stop) (void)hipEventDestroy(e);
        for (auto q : streams) (void)hipStreamDestroy(q);
        if (arena) (void)hipFree(arena);
        if (prof) (void)hipFree(prof);
        if (ord_arena) (void)hipFree(ord_arena);
        if (graph_arena) (void)hipFree(graph_arena);
    }
};

extern "C" int pt_universe_set_create(const pt_universe_job *jobs, int64_t n, int32_t model, int32_t p_norm,
                                      int32_t norm_flag, int32_t opt, int64_t bern, int64_t filter,
                                      pt_universe_set **out) {
    PT_CHECK(out && (jobs || n == 0), PT_EINVAL, "pt_universe_set_create: null argument");
    PT_CHECK(model == 0 || model == 1, PT_EINVAL, "model must be 0 (TransE) or 1 (TransH)");
    PT_CHECK(p_norm == 1 || p_norm == 2, PT_EINVAL, "p_norm must be 1 or 2");
    PT_CHECK(opt == PT_SGD || opt == PT_ADAGRAD, PT_EINVAL, "opt must be PT_SGD or PT_ADAGRAD");
    auto set = std::make_unique<pt_universe_set>();
    set->model = model; set->p_norm = p_norm; set->norm_flag = norm_flag; set->opt = opt;
    set->bern = bern; set->filter = filter;
    PT_HIP(hipGetDevice(&set->device));
    int64_t neg = -1;
    // layout of the per-universe workspace in one arena
    auto al = [](int64_t b) { return (b + 255) & ~int64_t(255); };
    struct Slot {
        int64_t states, contrib, grad, flags;
    };
    std::vector<Slot> slots((size_t)n);
    // every universe's LCG states first, 64 words each in set order (one upload, one reset copy)
    int64_t total = al(512 * std::max<int64_t>(n, 1));
    for (int64_t i = 0; i < n; ++i) {
        const pt_universe_job &J = jobs[i];
        PT_CHECK(J.graph && J.seeds && J.ent && J.rel, PT_EINVAL, "universe job: null graph / seeds / tables");
        PT_CHECK(model == 0 || J.normv, PT_EINVAL, "TransH universe job needs normv");
        PT_CHECK(opt == PT_SGD || (J.ent_acc && J.rel_acc && (model == 0 || J.norm_acc)), PT_EINVAL,
                 "Adagrad universe job needs accumulators");
        PT_CHECK(J.threads > 0 && J.threads <= 64, PT_EINVAL, "universe job: threads must be in [1, 64]");
        PT_CHECK(J.dim > 0 && pt::universe_shape_supported(J.dim, model), PT_EINVAL, "universe job: unsupported dim");
        PT_CHECK(J.batch_size >= 0 && J.epochs >= 0 && J.nbatches >= 0, PT_EINVAL, "universe job: negative sizes");
        PT_CHECK(neg < 0 || J.neg == neg, PT_EINVAL, "universe jobs must share neg");
        PT_CHECK(J.neg >= 1, PT_EINVAL, "universe job: neg must be >= 1");
        neg = J.neg;
        const pt::Graph &g = reinterpret_cast<const pt_graph *>(J.graph)->g;
        PT_CHECK(g.train_total > 0 || J.batch_size == 0, PT_EINVAL, "universe job: empty graph");
        PT_CHECK(J.batch_size * (4 + J.neg) <= 16384, PT_EINVAL, "universe job: batch too large for the LDS work list");
        const int64_t rows = g.ent_total + g.rel_total * (model == 1 ? 2 : 1);
        slots[i].contrib = total; total += al(4 * J.batch_size * (4 + J.neg) * J.dim);
        slots[i].grad = total;   total += al(4 * rows * J.dim);
        slots[i].flags = total;  total += al(4 * (g.ent_total + 2 * g.rel_total));
    }
    set->neg = neg < 0 ? 1 : neg;
    const int64_t us_off = total;
    total += al((int64_t)sizeof(pt::UniverseDev) * std::max<int64_t>(n, 1));
    const int64_t counter_off = total;
    total += al(sizeof(int) * 64);   // one work-queue counter per row shape
    PT_HIP(hipMalloc(&set->arena, (size_t)total));
    char *base = (char *)set->arena;
    PT_HIP(hipMemset(base, 0, (size_t)us_off));
    // LDS budget per universe workgroup: the device's per-workgroup limit, at most half a CU, minus the
    // kernel's static LDS. (The workgroups run one per CU at 256 VGPRs, but the whole CU's LDS measured
    // slower: C5 37.6 -> 352 ms, C4 104 -> 107 ms, C3 unchanged.)
    int max_lds = 64 << 10;
    (void)hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, set->device);
    const int64_t lds_budget = std::min<int64_t>(max_lds, 80 << 10) - 1024 - 2048;   // (2 KB: the static PreTables)
    // one persistent launch per row shape, its universes longest dependent step chain first (the work
    // queue then approximates longest-processing-time scheduling over the launch's workgroups)
    // A universe's time (the CU-share model and the queue order): steps x cycles per step, a fixed part plus a
    // per-positive part that grows with the padded row (lanes x floats per lane) - fitted to every universe's
    // measured cycles per step (r04, PT_UNI_PROF dumps of C3 and C4: 6,587 + bs x (63.3 + 0.681 x row slots);
    // residual spread 18 % / 14 %, against 21 % / 20 % for the earlier fixed + rounds-of-positives model)
    auto work = [&](int64_t i) {
        const int rs = pt::universe_shape_row_slots(pt::universe_shape_id(jobs[i].dim, model));
        return (double)jobs[i].epochs * (double)jobs[i].nbatches *
               (6587.0 + (double)std::max<int64_t>(jobs[i].batch_size, 1) * (63.3 + 0.681 * rs));
    };
    std::vector<int64_t> order((size_t)n);
    for (int64_t i = 0; i < n; ++i) order[i] = i;
    // Kernel (class) per universe: its row shape's class kernel, or - for up to three "hot" shapes of class 1
    // (TransE), those holding the set's longest universes - a kernel compiled for that shape alone. A class
    // kernel is register-allocated for all its shapes at once: the longest C3 universe's shape alone runs its
    // chain in 78 instead of 94 Mcycles. At most four launches in all (the hardware queues a process gets).
    std::vector<int> cls_v((size_t)n);
    std::vector<int> team_w;
    {
        std::vector<int> shape_v((size_t)n);
        std::map<int, double> hot_cost;   // class-1 shape -> its longest universe (steps x (4 + rounds))
        for (int64_t i = 0; i < n; ++i) {
            shape_v[i] = pt::universe_shape_id(jobs[i].dim, model);
            cls_v[i] = pt::universe_shape_class(shape_v[i]);
            if (model != PT_TRANSE || cls_v[i] != 1) continue;
            const int64_t gpb = pt::universe_shape_groups(shape_v[i], model);
            const double c = (double)jobs[i].epochs * (double)jobs[i].nbatches *
                             (4.0 + (double)((std::max<int64_t>(jobs[i].batch_size, 1) + gpb - 1) / gpb));
            hot_cost[shape_v[i]] = std::max(hot_cost[shape_v[i]], c);
        }
        std::vector<std::pair<double, int>> cand;
        for (auto &kv : hot_cost) cand.push_back({kv.second, kv.first});
        std::sort(cand.begin(), cand.end(), std::greater<std::pair<double, int>>());
        std::set<int> hot;
        for (auto &c : cand) {
            if (hot.size() >= 3) break;
            std::set<int> h2 = hot;
            h2.insert(c.second);
            std::set<int> launches;
            for (int64_t i = 0; i < n; ++i)
                launches.insert(h2.count(shape_v[i]) ? pt::kUniHotBase + shape_v[i] : cls_v[i]);
            if (launches.size() > 4) break;
            hot = h2;
        }
        if (const char *v = pt_tuning_env("PT_UNI_HOT"))   // tuning: 0 = class kernels only
            if (atoi(v) == 0) hot.clear();
        for (int64_t i = 0; i < n; ++i)
            if (hot.count(shape_v[i])) cls_v[i] = pt::kUniHotBase + shape_v[i];
        // Teams (universes_team.h): with fewer universes than CUs the set's makespan is its longest chain and CUs
        // idle. The spare CUs go, two at a time, to the universe whose modelled time is longest: its team doubles
        // (1 -> 2 -> 4 workgroups, modelled speed-ups kTeamSpeed), as long as a team universe's LDS plan fits and
        // at most two row shapes take teams (one launch per shape).
        int cus_t = 0;
        PT_HIP(hipDeviceGetAttribute(&cus_t, hipDeviceAttributeMultiprocessorCount, set->device));
        const int wmax = g_team_width.load();
        team_w.assign((size_t)n, 1);
        if (model == PT_TRANSE && wmax > 1 && n < cus_t) {
            static const double kTeamSpeed[5] = {0.0, 1.0, 1.6, 0.0, 2.4};
            std::vector<bool> ok((size_t)n, false);
            int64_t cap = 1;   // the set's work-list capacity (its largest batch)
            for (int64_t i = 0; i < n; ++i) cap = std::max<int64_t>(cap, jobs[i].batch_size * (4 + jobs[i].neg));
            for (int64_t i = 0; i < n; ++i)
                ok[i] = pt::universe_team_shape(shape_v[i], model) && jobs[i].batch_size > 0 &&
                        jobs[i].epochs * jobs[i].nbatches > 0;
            // the team launch's LDS with one presampled batch, over its universes' largest sizes (the launch gets as
            // many batches as then fit)
            int64_t m_rel = 0, m_ent = 0, m_slots = 0, m_seq = 0, m_rstep = 0, m_dim = 0;
            auto fits_with = [&](int64_t i) {
                const pt::Graph &g = reinterpret_cast<const pt_graph *>(jobs[i].graph)->g;
                const int64_t b = jobs[i].batch_size;
                return pt::universe_team_lds_bytes(cap, std::max(m_rel, g.rel_total), std::max(m_ent, g.ent_total),
                                                   std::max(m_slots, b * (2 + jobs[i].neg)),
                                                   1, std::max(m_seq, b * (1 + jobs[i].neg)),
                                                   std::max(m_rstep, std::min(b, g.rel_total)),
                                                   std::max(m_dim, jobs[i].dim)) <= lds_budget;
            };
            int64_t spare = (int64_t)cus_t - n;
            auto t_of = [&](int64_t i) { return work(i) / kTeamSpeed[team_w[(size_t)i]]; };
            while (spare > 0) {
                int64_t best = -1;
                for (int64_t i = 0; i < n; ++i)
                    if (best < 0 || t_of(i) > t_of(best)) best = i;
                if (best < 0 || !ok[best] || team_w[best] >= wmax) break;   // the longest cannot get faster
                const int64_t cost = team_w[best];
                if (cost > spare) break;
                std::set<int> shapes;
                for (int64_t i = 0; i < n; ++i)
                    if (team_w[i] > 1 || i == best) shapes.insert(shape_v[i]);
                if (shapes.size() > 2 || (team_w[best] == 1 && !fits_with(best))) break;
                if (team_w[best] == 1) {
                    const pt::Graph &g = reinterpret_cast<const pt_graph *>(jobs[best].graph)->g;
                    m_rel = std::max(m_rel, g.rel_total);
                    m_ent = std::max(m_ent, g.ent_total);
                    m_slots = std::max(m_slots, jobs[best].batch_size * (2 + jobs[best].neg));
                    m_seq = std::max(m_seq, jobs[best].batch_size * (1 + jobs[best].neg));
                    m_rstep = std::max(m_rstep, std::min(jobs[best].batch_size, g.rel_total));
                    m_dim = std::max(m_dim, jobs[best].dim);
                }
                team_w[best] *= 2;
                spare -= cost;
            }
            if (const char *v = pt_tuning_env("PT_UNI_TEAMS"))   // tuning: 0 = no teams
                if (atoi(v) == 0) team_w.assign((size_t)n, 1);
            for (int64_t i = 0; i < n; ++i)
                if (team_w[i] > 1) cls_v[i] = pt::kUniTeamBase + shape_v[i];
        }
    }
    auto cls_of = [&](int64_t i) { return cls_v[(size_t)i]; };
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        const int sa = cls_of(a), sb = cls_of(b);
        if (sa != sb) return sa < sb;
        return work(a) > work(b);
    });
    for (int64_t k = 0; k < n; ++k) {
        const int sh = cls_of(order[k]);
        if (set->groups.empty() || set->groups.back().shape != sh) set->groups.push_back({sh, k, 0, 0.0});
        set->groups.back().n += 1;
        set->groups.back().work += work(order[k]);
    }
    PT_CHECK(set->groups.size() <= 64, PT_EINVAL, "too many universe shape classes");
    // a team launch takes one CU per member of its universes
    auto is_team = [&](size_t k) { return set->groups[k].shape >= pt::kUniTeamBase; };
    for (size_t k = 0; k < set->groups.size(); ++k) {
        if (!is_team(k)) continue;
        int64_t w = 0;
        for (int64_t q = set->groups[k].off; q < set->groups[k].off + set->groups[k].n; ++q) w += team_w[order[q]];
        set->groups[k].share = w;
    }
    // CU shares: a universe's time by the step-cost model (`work`); give every group one CU,
    // then each further CU to the group whose LPT makespan over its current share is longest (the launches run
    // concurrently, so the slowest group ends the set)
    {
        int cus = 0;
        PT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, set->device));
        // (the step-cost model of `work`: with it the shares no longer leave C3's float4 hot launch ending 2 ms after
        // the longest universe, which the rounds-of-positives model did)
        std::vector<std::vector<double>> tg(set->groups.size());
        for (size_t k = 0; k < set->groups.size(); ++k) {
            const auto &gr = set->groups[k];
            for (int64_t q = gr.off; q < gr.off + gr.n; ++q) tg[k].push_back(work(order[q]));
            std::sort(tg[k].begin(), tg[k].end(), std::greater<double>());
        }
        auto makespan = [&](size_t k, int64_t s) {
            std::priority_queue<double, std::vector<double>, std::greater<double>> m;
            for (int64_t i = 0; i < s; ++i) m.push(0.0);
            double end = 0;
            for (double t : tg[k]) {
                const double f = m.top() + t;
                m.pop();
                m.push(f);
                end = std::max(end, f);
            }
            return end;
        };
        std::vector<double> ms(set->groups.size());
        int64_t left = (int64_t)cus;
        for (size_t k = 0; k < set->groups.size(); ++k) {
            ms[k] = makespan(k, 1);
            left -= set->groups[k].share;
        }
        for (; left > 0; --left) {
            size_t best = set->groups.size();
            for (size_t k = 0; k < set->groups.size(); ++k)
                if (!is_team(k) && set->groups[k].share < set->groups[k].n &&
                    (best == set->groups.size() || ms[k] > ms[best]))
                    best = k;
            if (best == set->groups.size()) break;
            set->groups[best].share += 1;
            ms[best] = makespan(best, set->groups[best].share);
        }
    }
    set->d_us = (pt::UniverseDev *)(base + us_off);
    set->d_counter = (int *)(base + counter_off);
    set->host.reserve((size_t)n);
    int64_t loss_off = 0;
    std::vector<int64_t> loss_of((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        loss_of[i] = loss_off;
        loss_off += jobs[i].epochs;
    }
    // the universes' device graphs: host images built on worker threads (each distinct graph once), placed in
    // one allocation with one copy
    std::vector<const pt::Graph *> uniq;
    std::vector<int64_t> gidx((size_t)n);
    {
        std::unordered_map<const pt::Graph *, int64_t> seen;
        for (int64_t i = 0; i < n; ++i) {
            const pt::Graph *gp = &reinterpret_cast<const pt_graph *>(jobs[i].graph)->g;
            auto it = seen.find(gp);
            if (it == seen.end()) {
                it = seen.emplace(gp, (int64_t)uniq.size()).first;
                uniq.push_back(gp);
            }
            gidx[i] = it->second;
        }
    }
    std::vector<std::vector<char>> images(uniq.size());
    {
        std::atomic<int64_t> next{0};
        auto work = [&]() {
            for (int64_t k; (k = next.fetch_add(1)) < (int64_t)uniq.size();)
                images[k] = const_cast<pt::Graph *>(uniq[k])->device_image();
        };
        const int64_t nw = std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
        std::vector<std::thread> pool;
        for (int64_t w = 1; w < std::min<int64_t>(nw, (int64_t)uniq.size()); ++w) pool.emplace_back(work);
        work();
        for (auto &th : pool) th.join();
    }
    std::vector<int64_t> goff(uniq.size() + 1, 0);
    for (size_t k = 0; k < uniq.size(); ++k) goff[k + 1] = goff[k] + al((int64_t)images[k].size());
    {
        std::vector<char> staging((size_t)std::max<int64_t>(goff.back(), 1));
        for (size_t k = 0; k < uniq.size(); ++k) memcpy(staging.data() + goff[k], images[k].data(), images[k].size());
        PT_HIP(hipMalloc(&set->graph_arena, staging.size()));
        PT_HIP(hipMemcpy(set->graph_arena, staging.data(), staging.size(), hipMemcpyHostToDevice));
    }
    int64_t max_bs = 0, max_relg = 0, max_ent = 0, max_rel = 0, max_seq = 0, max_nb = 0;
    set->seeds0.assign((size_t)(64 * std::max<int64_t>(n, 1)), 0);
    for (int64_t i : order) {
        const pt_universe_job &J = jobs[i];
        const pt::Graph &g = *uniq[(size_t)gidx[i]];
        const int64_t k = (int64_t)set->host.size();   // position in the set
        pt::UniverseDev U{};
        U.g = g.bind_image((char *)set->graph_arena + goff[(size_t)gidx[i]]);
        U.states = (uint64_t *)(base + 512 * k);
        std::copy(J.seeds, J.seeds + J.threads, set->seeds0.begin() + 64 * k);
        U.ent = J.ent; U.rel = J.rel; U.normv = J.normv;
        U.ent_acc = J.ent_acc; U.rel_acc = J.rel_acc; U.norm_acc = J.norm_acc;
        float *gr = (float *)(base + slots[i].grad);
        U.gent = gr;
        U.grel = gr + g.ent_total * J.dim;
        U.gnorm = model == 1 ? U.grel + g.rel_total * J.dim : nullptr;
        int32_t *fl = (int32_t *)(base + slots[i].flags);
        U.fent = fl;
        U.frel = fl + g.ent_total;
        U.fnorm = U.frel + g.rel_total;
        U.contrib = (float *)(base + slots[i].contrib);
        U.losses = nullptr;
        U.prof = nullptr;   // pt_universe_set_profiling
        U.threads = J.threads; U.bs = J.batch_size; U.nbatches = J.nbatches; U.epochs = J.epochs; U.dim = J.dim;
        U.lr = J.lr; U.margin = J.margin;
        U.shape = pt::universe_shape_id(J.dim, model);
        if (set->host_of_job.empty()) set->host_of_job.assign((size_t)n, -1);
        set->host_of_job[(size_t)i] = (int64_t)set->host.size();
        set->host.push_back(U);
        set->host_team_w.push_back(team_w.empty() ? 1 : team_w[(size_t)i]);
        set->host_loss_off.push_back(loss_of[i]);
        max_bs = std::max(max_bs, J.batch_size);
        max_relg = std::max(max_relg, g.rel_total * J.dim);
        max_ent = std::max(max_ent, g.ent_total);
        max_rel = std::max(max_rel, g.rel_total);
        max_seq = std::max(max_seq, J.batch_size * (1 + J.neg));
        max_nb = std::max(max_nb, J.nbatches);
    }
    if (n > 0) PT_HIP(hipMemcpy(base, set->seeds0.data(), 8 * set->seeds0.size(), hipMemcpyHostToDevice));
    // LDS plan (within the device's per-workgroup limit and half a CU): the work list is required;
    // then, each if it still fits, the relation gradient rows (the contended rows of the scatter), the
    // entity contribution lists (replace the entity float atomics), the touched flags, and as many
    // presampled batches as fit
    auto &C = set->cfg;
    C.list_cap = std::max<int64_t>(max_bs * (4 + set->neg), 1);
    auto a4 = [](int64_t v) { return 4 * ((v + 3) & ~int64_t(3)); };
    const int64_t list_b = a4(C.list_cap);
    const int64_t relg_b = 4 * max_relg * (model == 1 ? 2 : 1);
    int64_t used = list_b;
    auto env_on = [](const char *name) {
        const char *v = pt_tuning_env(name);
        return !v || atoi(v) != 0;
    };
    PT_CHECK(used <= lds_budget, PT_EINVAL, "universe batch too large for the LDS work list");
    const int64_t per_batch = 12 * max_seq;
    // entity rows as contribution lists (heads for entities and relations, next per slot)
    const int64_t heads_b = a4(max_ent + 2 * max_rel) + a4(max_bs * (4 + set->neg));
    C.contrib = used + heads_b <= lds_budget && env_on("PT_UNI_CONTRIB");
    used += C.contrib ? heads_b : 0;
    // relation rows: LDS gradient rows (hot rows, few) if they fit, else contribution lists
    C.lds_relgrad = used + relg_b <= lds_budget && env_on("PT_UNI_RELGRAD");
    C.rel_list = C.contrib && !C.lds_relgrad;
    used += C.lds_relgrad ? relg_b : 0;
    // touched flags of the rows that are not lists
    const int64_t nfl = (C.contrib ? 0 : max_ent) + (C.rel_list ? 0 : 2 * max_rel);
    const int64_t flags_b = a4(nfl);
    C.lds_flags = nfl > 0 && used + flags_b <= lds_budget && env_on("PT_UNI_LDSFLAGS");
    used += C.lds_flags ? flags_b : 0;
    C.pchunk = env_on("PT_UNI_PRESAMPLE") && per_batch > 0 ? std::min<int64_t>(max_nb, (lds_budget - used) / per_batch)
                                                            : 0;
    if (C.pchunk < 0) C.pchunk = 0;
    used += C.pchunk * per_batch;
    C.lds_bytes = used;
    // agent-scope fences only while some gradient row is a global float atomic (or a flag global)
    C.agent_fence = !(C.contrib && (C.rel_list || (C.lds_relgrad && C.lds_flags)));
    if (const char *v = pt_tuning_env("PT_UNI_FENCE")) C.agent_fence = C.agent_fence || atoi(v) != 0;
    C.threads = 512;
    // tuning overrides (benchmarks): PT_UNI_RELGRAD / CONTRIB / LDSFLAGS / PRESAMPLE = 0 disable the
    // LDS placements above, PT_UNI_FENCE=1 forces agent-scope fences
    // Team launches (universes_team.h): their LDS plan (every universe's presampled batches, as many as fit), one
    // arena for the relation / loss partials and arrival counters of their universes and the launch maps, each team's
    // members on blocks of one residue mod 8 (the dispatcher's round-robin over the XCDs: one L2 for the team -
    // performance only, the protocol does not depend on it)
    {
        int64_t t_rel = 0, t_ent = 0, t_slots = 0, t_seq = 0, t_nb = 0, t_rstep = 0, t_dim = 0, part_b = 0, n_team = 0,
                map_b = 0;
        // a team universe's partials: [W][R][D] relation rows, [W][epochs] losses, [W] XCD ids
        auto part_bytes = [&](const pt::UniverseDev &U, int w) {
            return al(4 * (w * U.g.rel_total * U.dim + w * U.epochs + w));
        };
        std::vector<int64_t> grid_of(set->groups.size(), 0);
        std::vector<std::vector<int32_t>> maps(set->groups.size());
        for (size_t k = 0; k < set->groups.size(); ++k) {
            const auto &gr = set->groups[k];
            if (gr.shape < pt::kUniTeamBase) continue;
            std::vector<std::pair<int, int64_t>> teams;   // (members, index from off)
            for (int64_t q = gr.off; q < gr.off + gr.n; ++q) {
                const pt::UniverseDev &U = set->host[(size_t)q];
                const int w = set->host_team_w[(size_t)q];
                teams.push_back({w, q - gr.off});
                t_rel = std::max(t_rel, U.g.rel_total);
                t_ent = std::max(t_ent, U.g.ent_total);
                t_slots = std::max(t_slots, U.bs * (2 + set->neg));
                t_seq = std::max(t_seq, U.bs * (1 + set->neg));
                t_nb = std::max(t_nb, U.nbatches);
                t_rstep = std::max(t_rstep, std::min(U.bs, U.g.rel_total));
                t_dim = std::max(t_dim, U.dim);
                part_b += part_bytes(U, w);
                ++n_team;
            }
            std::stable_sort(teams.begin(), teams.end(), [](const std::pair<int, int64_t> &a,
                                                            const std::pair<int, int64_t> &b) { return a.first > b.first; });
            int64_t used[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            std::vector<std::pair<int64_t, std::pair<int32_t, int32_t>>> blocks;
            for (const auto &t : teams) {
                int x = 0;
                for (int c = 1; c < 8; ++c)
                    if (used[c] < used[x]) x = c;
                for (int m = 0; m < t.first; ++m) blocks.push_back({x + 8 * (used[x] + m), {(int32_t)t.second, m}});
                used[x] += t.first;
            }
            int64_t rows = 0;
            for (int c = 0; c < 8; ++c) rows = std::max(rows, used[c]);
            grid_of[k] = 8 * rows;
            maps[k].assign((size_t)(2 * grid_of[k]), -1);
            for (const auto &b : blocks) {
                maps[k][(size_t)(2 * b.first)] = b.second.first;
                maps[k][(size_t)(2 * b.first + 1)] = b.second.second;
            }
            map_b += al(4 * (int64_t)maps[k].size());
        }
        if (n_team > 0) {
            auto &T = set->team_cfg;
            T = C;
            const int64_t fixed = pt::universe_team_lds_bytes(C.list_cap, t_rel, t_ent, t_slots, 0, t_seq, t_rstep, t_dim);
            T.pchunk = std::min<int64_t>(t_nb, (lds_budget - fixed) / std::max<int64_t>(12 * t_seq, 1));
            PT_CHECK(T.pchunk >= 1, PT_EINVAL, "team universes: LDS plan does not fit");
            T.lds_bytes = pt::universe_team_lds_bytes(C.list_cap, t_rel, t_ent, t_slots, T.pchunk, t_seq, t_rstep, t_dim);
            const int64_t sync_b = al(4 * (n_team + 1));   // + the error word
            const int64_t teams_b = al((int64_t)sizeof(pt::TeamDev) * (int64_t)set->host.size());
            PT_HIP(hipMalloc(&set->team_arena, (size_t)(part_b + sync_b + map_b + teams_b)));
            char *tb = (char *)set->team_arena;
            set->d_team_sync = (uint32_t *)(tb + part_b);
            set->n_team_sync = n_team;
            int64_t po = 0, si = 0, mo = part_b + sync_b;
            std::vector<pt::TeamDev> th(set->host.size(), pt::TeamDev{nullptr, nullptr, nullptr, 1});
            for (size_t k = 0; k < set->groups.size(); ++k) {
                auto &gr = set->groups[k];
                if (gr.shape < pt::kUniTeamBase) continue;
                for (int64_t q = gr.off; q < gr.off + gr.n; ++q) {
                    pt::TeamDev &T = th[(size_t)q];
                    T.w = set->host_team_w[(size_t)q];
                    T.part = (float *)(tb + po);
                    po += part_bytes(set->host[(size_t)q], T.w);
                    T.sync = set->d_team_sync + si++;
                    T.err = set->d_team_sync + n_team;
                }
                gr.d_map = (int32_t *)(tb + mo);
                gr.grid = grid_of[k];
                PT_HIP(hipMemcpy(gr.d_map, maps[k].data(), 4 * maps[k].size(), hipMemcpyHostToDevice));
                mo += al(4 * (int64_t)maps[k].size());
            }
            set->d_teams = (pt::TeamDev *)(tb + mo);
            PT_HIP(hipMemcpy(set->d_teams, th.data(), sizeof(pt::TeamDev) * th.size(), hipMemcpyHostToDevice));
        }
    }
    *out = set.release();
    return PT_OK;
}

extern "C" int pt_universe_set_deterministic(pt_universe_set *set, int32_t on) {
    PT_CHECK(set, PT_EINVAL, "null universe set");
    // the set enters reference-order mode only once its workspace exists: a failed call leaves the mode as it
    // was (a later train call then runs the fast kernel, never the ordered one without its arena)
    if (!on || set->host.empty() || set->ord_arena) {
        set->ordered = on != 0;
        return PT_OK;
    }
    auto al = [](int64_t b) { return (b + 255) & ~int64_t(255); };
    int64_t total = 0, max_seq = 0;
    std::vector<int64_t> off(set->host.size());
    for (size_t i = 0; i < set->host.size(); ++i) {
        const pt::UniverseDev &U = set->host[i];
        const int64_t seq = U.bs * (1 + set->neg);
        off[i] = total;
        total += al(16 * seq * U.dim);
        max_seq = std::max(max_seq, seq);
    }
    // the launch's LDS (dynamic plan + the kernel's static variables) against the per-workgroup limit
    int blk_lds = 64 << 10;
    (void)hipDeviceGetAttribute(&blk_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, set->device);
    size_t static_lds = 0;
    PT_HIP(pt::ordered_universe_static_lds(&static_lds));
    PT_CHECK(pt::ordered_universe_lds_bytes(max_seq) + (int64_t)static_lds <= (int64_t)blk_lds, PT_ENOTSUP,
             "reference-order mode: universe batch too large for the LDS plan");
    void *arena = nullptr;
    PT_HIP(hipMalloc(&arena, (size_t)std::max<int64_t>(total, 256)));
    set->ord_arena = arena;
    for (size_t i = 0; i < set->host.size(); ++i) set->host[i].ord = (float *)((char *)set->ord_arena + off[i]);
    set->ord_max_seq = max_seq;
    set->ordered = true;
    return PT_OK;
}

extern "C" int pt_universe_set_train(pt_universe_set *set, float *d_losses, void *stream) {
    PT_CHECK(set, PT_EINVAL, "null universe set");
    if (set->host.empty()) return PT_OK;
    hipStream_t st = (hipStream_t)stream;
    for (size_t i = 0; i < set->host.size(); ++i)
        set->host[i].losses = d_losses ? d_losses + set->host_loss_off[i] : nullptr;
    PT_HIP(hipMemcpyAsync(set->d_us, set->host.data(), sizeof(pt::UniverseDev) * set->host.size(),
                          hipMemcpyHostToDevice, st));
    if (set->ordered) {
        int cus = 0;
        PT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, set->device));
        const hipError_t e = pt::launch_universes_ordered(set->d_us, (int64_t)set->host.size(), set->d_counter, cus,
                                                          set->model, set->p_norm, set->norm_flag, set->opt, set->neg,
                                                          (int)set->bern, (int)set->filter, set->ord_max_seq, st);
        if (e != hipSuccess) return pt::fail(PT_EHIP, std::string("launch_universes_ordered: ") + hipGetErrorString(e));
        PT_HIP(hipStreamSynchronize(st));
        return PT_OK;
    }
    // one launch per shape class, concurrently, each over its share of the CUs (set at creation): forked from `st`
    // onto the process's class streams (each on a hardware queue of its own, class_streams) and joined back, so
    // the launches overlap whatever streams the caller's process already holds
    const size_t ng = set->groups.size();
    const int smode = class_stream_mode();
    std::vector<hipStream_t> qs(ng);
    if (smode == 0) {   // round 4's scheme (tuning A/B): class 0 on `st`, the others on per-set side streams
        while (set->streams.size() + 1 < ng) {
            hipStream_t q;
            PT_HIP(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
            set->streams.push_back(q);
        }
        for (size_t k = 0; k < ng; ++k) qs[k] = k == 0 ? st : set->streams[k - 1];
    } else {
        PT_HIP(class_streams(set->device, smode, ng, &qs));
    }
    while (set->events.size() < ng + 1) {
        hipEvent_t ev;
        PT_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        set->events.push_back(ev);
    }
    while (set->t_start.size() < ng) {
        hipEvent_t a, b;
        PT_HIP(hipEventCreate(&a));
        PT_HIP(hipEventCreate(&b));
        set->t_start.push_back(a);
        set->t_stop.push_back(b);
    }
    if (set->n_team_sync > 0) PT_HIP(hipMemsetAsync(set->d_team_sync, 0, 4 * (set->n_team_sync + 1), st));
    PT_HIP(hipEventRecord(set->events[0], st));
    for (size_t k = 0; k < ng; ++k)
        if (qs[k] != st) PT_HIP(hipStreamWaitEvent(qs[k], set->events[0], 0));
    for (size_t k = 0; k < ng; ++k) {
        const auto &gr = set->groups[k];
        const int64_t share = gr.share;
        hipStream_t q = qs[k];
        PT_HIP(hipEventRecord(set->t_start[k], q));
        // PT_UNI_GRID=1 (tuning): one workgroup per universe in every launch, the hardware dispatcher
        // interleaving the class launches as CUs free up, instead of a CU share per launch
        static const bool per_universe = [] {
            const char *v = pt_tuning_env("PT_UNI_GRID");
            return v && atoi(v) != 0;
        }();
        if (gr.shape >= pt::kUniTeamBase) {
            const hipError_t e = pt::launch_universes_team(set->d_us + gr.off, set->d_teams + gr.off, gr.d_map, gr.grid,
                                                           gr.shape - pt::kUniTeamBase, set->p_norm, set->norm_flag,
                                                           set->opt, set->neg, (int)set->bern, (int)set->filter,
                                                           set->team_cfg, q);
            if (e != hipSuccess) return pt::fail(PT_EHIP, std::string("launch_universes_team: ") + hipGetErrorString(e));
            PT_HIP(hipEventRecord(set->t_stop[k], q));
            continue;
        }
        const hipError_t e = pt::launch_universes(set->d_us + gr.off, gr.n, set->d_counter + k, gr.shape,
                                                  per_universe ? gr.n : share,
                                                  set->model, set->p_norm, set->norm_flag, set->opt, set->neg,
                                                  (int)set->bern, (int)set->filter, set->cfg, q);
        if (e != hipSuccess) return pt::fail(PT_EHIP, std::string("launch_universes: ") + hipGetErrorString(e));
        PT_HIP(hipEventRecord(set->t_stop[k], q));
    }
    for (size_t k = 0; k < ng; ++k) {
        if (qs[k] == st) continue;
        PT_HIP(hipEventRecord(set->events[k + 1], qs[k]));
        PT_HIP(hipStreamWaitEvent(st, set->events[k + 1], 0));
    }
    // the host array must outlive the async copy: this call returns only after it has been consumed
    PT_HIP(hipStreamSynchronize(st));
    set->timed = true;
    if (set->n_team_sync > 0) {
        uint32_t err = 0;
        PT_HIP(hipMemcpy(&err, set->d_team_sync + set->n_team_sync, 4, hipMemcpyDeviceToHost));
        PT_CHECK(err == 0, PT_EHIP, "team universes: a team member never arrived (workgroups not co-resident)");
    }
    return PT_OK;
}

// the class launches of the last fast-path train call: per launch its start and end (ms after the earliest start,
// HIP events on the launch's stream) and its universe count; the launches overlap when they run concurrently
extern "C" int pt_universe_set_launch_times(pt_universe_set *set, int64_t cap, float *out, int64_t *n_out) {
    PT_CHECK(set && n_out, PT_EINVAL, "pt_universe_set_launch_times: null argument");
    const int64_t ng = set->timed ? (int64_t)set->groups.size() : 0;
    *n_out = ng;
    if (!out || ng == 0) return PT_OK;
    PT_CHECK(cap >= ng, PT_EINVAL, "pt_universe_set_launch_times: cap below the launch count");
    for (int64_t k = 0; k < ng; ++k) {
        float a = 0.f, b = 0.f;
        PT_HIP(hipEventElapsedTime(&a, set->t_start[0], set->t_start[(size_t)k]));
        PT_HIP(hipEventElapsedTime(&b, set->t_start[0], set->t_stop[(size_t)k]));
        out[3 * k] = a;
        out[3 * k + 1] = b;
        out[3 * k + 2] = (float)set->groups[(size_t)k].n;
    }
    float lo = out[0];
    for (int64_t k = 1; k < ng; ++k) lo = std::min(lo, out[3 * k]);
    for (int64_t k = 0; k < ng; ++k) {
        out[3 * k] -= lo;
        out[3 * k + 1] -= lo;
    }
    return PT_OK;
}

// how the set trains: universes in team launches and the workgroups (CUs) those take
extern "C" int pt_universe_set_teams(const pt_universe_set *set, int64_t *team_universes, int64_t *team_workgroups) {
    PT_CHECK(set && team_universes && team_workgroups, PT_EINVAL, "pt_universe_set_teams: null argument");
    *team_universes = 0;
    *team_workgroups = 0;
    for (const auto &gr : set->groups)
        if (gr.shape >= pt::kUniTeamBase) {
            *team_universes += gr.n;
            *team_workgroups += gr.share;
        }
    return PT_OK;
}

// the sampler streams back to the jobs' creation states (a benchmark re-runs the same training from the same
// start: the caller restores the tables and optimizer state)
// whether universes of this dim train on the fast path (its row shape is compiled into its class kernel)
extern "C" int pt_universe_dim_supported(int64_t dim, int32_t model) {
    return (model == PT_TRANSE || model == PT_TRANSH) && pt::universe_shape_supported(dim, model) ? 1 : 0;
}

extern "C" int pt_universe_set_reset(pt_universe_set *set) {
    PT_CHECK(set, PT_EINVAL, "null universe set");
    if (!set->host.empty())   // the states block at the arena's start, in set order
        PT_HIP(hipMemcpy(set->arena, set->seeds0.data(), 8 * set->seeds0.size(), hipMemcpyHostToDevice));
    return PT_OK;
}

extern "C" int pt_universe_set_states(pt_universe_set *set, int64_t job, uint64_t *out) {
    PT_CHECK(set && out, PT_EINVAL, "pt_universe_set_states: null argument");
    PT_CHECK(job >= 0 && job < (int64_t)set->host_of_job.size(), PT_EINVAL, "pt_universe_set_states: bad job index");
    const pt::UniverseDev &U = set->host[(size_t)set->host_of_job[(size_t)job]];
    PT_HIP(hipDeviceSynchronize());
    PT_HIP(hipMemcpy(out, U.states, sizeof(uint64_t) * (size_t)U.threads, hipMemcpyDeviceToHost));
    return PT_OK;
}

// per-universe cycle counters of the fast kernel (clock64 around its phases), off by default
extern "C" int pt_universe_set_profiling(pt_universe_set *set, int32_t on) {
    PT_CHECK(set, PT_EINVAL, "null universe set");
    if (on && !set->prof && !set->host.empty()) {
        PT_HIP(hipMalloc((void **)&set->prof, 512 * set->host.size()));
        PT_HIP(hipMemset(set->prof, 0, 512 * set->host.size()));
    }
    for (size_t i = 0; i < set->host.size(); ++i) set->host[i].prof = on && set->prof ? set->prof + 64 * i : nullptr;
    return PT_OK;
}

// diagnostics: per universe (set order) 64 words: cycles in presampling / phase A / phase B, steps, batch size,
// dim, entities, start / duration (100 MHz wall clock) of the last train call with profiling on; team universes: word
// 60 (team width << 32 | one XCD), word 61 the cycles in team barriers; word 62 the rows
// updated in phase B summed over the steps; the other words 8-63 phase stamps of one step (tuning build)
extern "C" int pt_universe_set_profile(pt_universe_set *set, uint64_t *out) {
    PT_CHECK(set && out, PT_EINVAL, "null argument");
    PT_CHECK(set->prof, PT_ESTATE, "profiling not enabled (pt_universe_set_profiling)");
    PT_HIP(hipDeviceSynchronize());
    PT_HIP(hipMemcpy(out, set->prof, 512 * set->host.size(), hipMemcpyDeviceToHost));
    return PT_OK;
}

extern "C" int pt_universe_set_free(pt_universe_set *set) {
    if (set) (void)hipDeviceSynchronize();
    delete set;
    return PT_OK;
}

extern "C" int pt_universes_train_ex(const pt_universe_job *jobs, int64_t n, int32_t model, int32_t p_norm,
                                     int32_t norm_flag, int32_t opt, int64_t bern, int64_t filter, int32_t flags,
                                     float *d_losses, void *stream) {
    PT_CHECK((flags & ~PT_DETERMINISTIC) == 0, PT_EINVAL, "pt_universes_train_ex: unknown flags");
    pt_universe_set *set = nullptr;
    int rc = pt_universe_set_create(jobs, n, model, p_norm, norm_flag, opt, bern, filter, &set);
    if (rc) return rc;
    if (flags & PT_DETERMINISTIC) rc = pt_universe_set_deterministic(set, 1);
    if (!rc) rc = pt_universe_set_train(set, d_losses, stream);
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    pt_universe_set_free(set);
    if (!rc && e != hipSuccess) rc = pt::fail(PT_EHIP, std::string("pt_universes_train: ") + hipGetErrorString(e));
    return rc;
}

// initial universe tables, torch-CPU-generator-identical (torch_init.hip)
extern "C" int pt_torch_init_tables(const pt_torch_init_job *jobs, int64_t n, void *stream) {
    PT_CHECK(n >= 0 && (jobs || n == 0), PT_EINVAL, "pt_torch_init_tables: null jobs");
    if (n == 0) return PT_OK;
    for (int64_t i = 0; i < n; ++i) {
        const pt_torch_init_job &J = jobs[i];
        PT_CHECK(J.ntab >= 0 && J.ntab <= 4 && J.skip >= 0, PT_EINVAL, "pt_torch_init_tables: bad job");
        for (int k = 0; k < J.ntab; ++k)
            PT_CHECK(J.numel[k] >= 0 && (J.out[k] || J.numel[k] == 0), PT_EINVAL, "pt_torch_init_tables: null table");
    }
    hipStream_t st = (hipStream_t)stream;
    pt_torch_init_job *d = nullptr;
    PT_HIP(hipMallocAsync((void **)&d, sizeof(pt_torch_init_job) * (size_t)n, st));
    hipError_t e = hipMemcpyAsync(d, jobs, sizeof(pt_torch_init_job) * (size_t)n, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = pt::launch_torch_init(d, n, st);
    const hipError_t f = hipFreeAsync(d, st);
    const hipError_t w = hipStreamSynchronize(st);   // the caller's job array may go away on return
    if (e == hipSuccess) e = f != hipSuccess ? f : w;
    if (e != hipSuccess) return pt::fail(PT_EHIP, std::string("pt_torch_init_tables: ") + hipGetErrorString(e));
    return PT_OK;
}

extern "C" int pt_universes_train(const pt_universe_job *jobs, int64_t n, int32_t model, int32_t p_norm,
                                  int32_t norm_flag, int32_t opt, int64_t bern, int64_t filter, float *d_losses,
                                  void *stream) {
    pt_universe_set *set = nullptr;
    int rc = pt_universe_set_create(jobs, n, model, p_norm, norm_flag, opt, bern, filter, &set);
    if (rc) return rc;
    rc = pt_universe_set_train(set, d_losses, stream);
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    pt_universe_set_free(set);
    if (!rc && e != hipSuccess) rc = pt::fail(PT_EHIP, std::string("pt_universes_train: ") + hipGetErrorString(e));
    return rc;
}

// ======================================================================== link prediction =======
extern "C" int pt_lp_min_scores(const pt_lp_universe *us, int64_t n_universes, int32_t model, int32_t p_norm,
                                int32_t norm_flag, const pt_lp_pair *pairs, int64_t n_pairs,
                                int64_t global_ent_total, float *d_key_rows, float *d_key_tuple, void *stream) {
    PT_CHECK((us && pairs && d_key_rows) || n_pairs == 0, PT_EINVAL, "pt_lp_min_scores: null argument");
    if (n_pairs == 0) return PT_OK;
    hipStream_t st = (hipStream_t)stream;
    // per universe once: its dim's row shape is instantiated, and the job key of that shape (below)
    auto shape_key = [](int64_t dim) {
        const pt::Shape s = pt::pick_shape(dim);
        return (int64_t)s.G * 10000 + (int64_t)s.VEC * 100 + s.KCH;
    };
    std::vector<int64_t> u_shape((size_t)n_universes, -1);
    for (int64_t u = 0; u < n_universes; ++u)
        if (pt::shape_supported(us[u].dim)) u_shape[(size_t)u] = shape_key(us[u].dim);
    for (int64_t i = 0; i < n_pairs; ++i) {
        const pt_lp_pair &p = pairs[i];
        PT_CHECK(p.universe >= 0 && p.universe < n_universes, PT_EINVAL, "pair universe out of range");
        const pt_lp_universe &U = us[p.universe];
        PT_CHECK(p.anchor >= 0 && p.anchor < U.ent_total && p.rel >= 0 && p.rel < U.rel_total, PT_EINVAL,
                 "pair local ids out of range");
        PT_CHECK(p.side == 0 || p.side == 1, PT_EINVAL, "pair side must be 0 or 1");
        PT_CHECK(p.key >= 0, PT_EINVAL, "pair key must be non-negative");
        PT_CHECK(u_shape[(size_t)p.universe] >= 0, PT_ENOTSUP, "dim not supported");
    }
    // Jobs = (lane-group row shape of the universes' dims, key batch): one launch pair per job covers every
    // dim of that shape (C3's ~80 dims take ~10 shapes: one launch pair per dim left most of the GPU idle). A
    // key batch's score rows (keys x global_ent_total floats) are sized to stay resident in the Infinity
    // Cache while its pairs' atomicMins land (PT_LP_BATCH_MB, default 192); inside a job the pairs are
    // sorted by universe so each universe's entity rows are read once per job.
    int64_t n_keys = 0;
    for (int64_t i = 0; i < n_pairs; ++i) n_keys = std::max<int64_t>(n_keys, (int64_t)pairs[i].key + 1);
    int64_t batch_mb = 192;
    if (const char *v = pt_tuning_env("PT_LP_BATCH_MB")) batch_mb = std::max<int64_t>(1, atoll(v));
    const int64_t keys_per_batch =
        std::max<int64_t>(1, (batch_mb << 20) / (4 * std::max<int64_t>(global_ent_total, 1)));
    const int64_t n_batches = (n_keys + keys_per_batch - 1) / keys_per_batch;
    // jobs ordered by (shape key, batch); the pairs of a (job, universe) keep their input order: a counting sort
    // over (job, universe) in place of per-job per-universe vectors (2 M pairs for C4)
    std::vector<int64_t> shapes(u_shape);
    std::sort(shapes.begin(), shapes.end());
    shapes.erase(std::unique(shapes.begin(), shapes.end()), shapes.end());
    std::vector<int32_t> u_si((size_t)n_universes);
    for (int64_t u = 0; u < n_universes; ++u)
        u_si[(size_t)u] = (int32_t)(std::lower_bound(shapes.begin(), shapes.end(), u_shape[(size_t)u]) - shapes.begin());
    const int64_t n_jobs = (int64_t)shapes.size() * n_batches;
    auto job_of = [&](const pt_lp_pair &p) { return (int64_t)u_si[(size_t)p.universe] * n_batches + p.key / keys_per_batch; };
    std::vector<int64_t> cnt((size_t)(n_jobs * n_universes + 1), 0);
    for (int64_t i = 0; i < n_pairs; ++i) ++cnt[(size_t)(job_of(pairs[i]) * n_universes + pairs[i].universe + 1)];
    for (size_t c = 1; c < cnt.size(); ++c) cnt[c] += cnt[c - 1];
    std::vector<pt::LpPair> hp((size_t)n_pairs);
    {
        std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
        for (int64_t i = 0; i < n_pairs; ++i) {
            const pt_lp_pair &p = pairs[i];
            hp[(size_t)fill[(size_t)(job_of(p) * n_universes + p.universe)]++] =
                pt::LpPair{p.key, p.universe, p.anchor, p.rel, p.side};
        }
    }
    std::vector<pt::LpUniverseDev> hu((size_t)n_universes);
    for (int64_t i = 0; i < n_universes; ++i)
        hu[i] = pt::LpUniverseDev{us[i].ent, us[i].rel, us[i].normv, us[i].d_ent_remap, us[i].ent_total, us[i].dim};
    // host staging, kept alive until the stream has consumed it (synchronize at the end). Per job: its
    // pairs contiguous and sorted by universe; uoff[job][2u], uoff[job][2u+1] = universe u's range
    // relative to the job's first pair
    std::vector<int64_t> uoff;
    std::vector<int32_t> uids;
    struct DimJob {
        int64_t dim, p_begin, p_end, u_begin, u_end, max_ent, uoff_begin;
    };
    std::vector<DimJob> dj;
    for (int64_t j = 0; j < n_jobs; ++j) {
        const int64_t b0 = cnt[(size_t)(j * n_universes)], b1 = cnt[(size_t)((j + 1) * n_universes)];
        if (b1 == b0) continue;
        DimJob d{0, b0, b1, (int64_t)uids.size(), 0, 0, (int64_t)uoff.size()};   // dim: the largest
        uoff.resize(uoff.size() + 2 * (size_t)n_universes, 0);
        for (int64_t u = 0; u < n_universes; ++u) {
            const int64_t lo = cnt[(size_t)(j * n_universes + u)], hi = cnt[(size_t)(j * n_universes + u + 1)];
            if (hi == lo) continue;
            uoff[d.uoff_begin + 2 * u] = lo - b0;
            uoff[d.uoff_begin + 2 * u + 1] = hi - b0;
            uids.push_back((int32_t)u);
            d.max_ent = std::max(d.max_ent, us[u].ent_total);
            d.dim = std::max(d.dim, us[u].dim);
        }
        d.u_end = (int64_t)uids.size();
        dj.push_back(d);
    }
    int64_t max_dim = 0;
    for (auto &d : dj) max_dim = std::max(max_dim, d.dim);
    max_dim = (max_dim + 3) & ~int64_t(3);   // every job's scratch region 16-byte aligned (float4 rows)
    const size_t scratch = (size_t)n_pairs * (size_t)max_dim * (model == 1 ? 2 : 1);
    char *blk = nullptr;
    const size_t bytes = sizeof(pt::LpUniverseDev) * hu.size() + sizeof(pt::LpPair) * hp.size() +
                         sizeof(int64_t) * uoff.size() + sizeof(int32_t) * (uids.size() + 1) + sizeof(float) * scratch +
                         5 * 256;
    PT_HIP(hipMallocAsync((void **)&blk, bytes, st));
    auto carve = [&](size_t n) {
        char *p = blk;
        blk += (n + 255) & ~size_t(255);
        return p;
    };
    char *base0 = blk;
    auto *du = (pt::LpUniverseDev *)carve(sizeof(pt::LpUniverseDev) * hu.size());
    auto *dp = (pt::LpPair *)carve(sizeof(pt::LpPair) * hp.size());
    auto *duoff = (int64_t *)carve(sizeof(int64_t) * uoff.size());
    auto *duids = (int32_t *)carve(sizeof(int32_t) * (uids.size() + 1));
    auto *dbase = (float *)carve(sizeof(float) * scratch);
    PT_HIP(hipMemcpyAsync(du, hu.data(), sizeof(pt::LpUniverseDev) * hu.size(), hipMemcpyHostToDevice, st));
    PT_HIP(hipMemcpyAsync(dp, hp.data(), sizeof(pt::LpPair) * hp.size(), hipMemcpyHostToDevice, st));
    PT_HIP(hipMemcpyAsync(duoff, uoff.data(), sizeof(int64_t) * uoff.size(), hipMemcpyHostToDevice, st));
    PT_HIP(hipMemcpyAsync(duids, uids.data(), sizeof(int32_t) * uids.size(), hipMemcpyHostToDevice, st));
    int rc = PT_OK;
    for (auto &d : dj) {
        const int64_t np = d.p_end - d.p_begin;
        float *b = dbase + d.p_begin * max_dim * (model == 1 ? 2 : 1);   // the group's own scratch region
        float *nrm = model == 1 ? b + np * d.dim : nullptr;
        const hipError_t e = pt::launch_lp_min(du, dp + d.p_begin, np, duoff + d.uoff_begin, duids + d.u_begin,
                                               d.u_end - d.u_begin,
                                               d.dim, d.max_ent, model, p_norm, norm_flag, global_ent_total,
                                               d.dim, b, nrm, d_key_rows, d_key_tuple, st);
        if (e != hipSuccess) {
            rc = pt::fail(PT_EHIP, std::string("launch_lp_min: ") + hipGetErrorString(e));
            break;
        }
    }
    (void)hipFreeAsync(base0, st);
    PT_HIP(hipStreamSynchronize(st));   // host vectors above must outlive the async copies
    return rc;
}

extern "C" int pt_rank_rows(const float *d_rows, int64_t ent_total, const int64_t *d_row_of, const int64_t *d_truth,
                            const float *d_repl, const int64_t *d_part_off, const int64_t *d_part, int64_t n,
                            int64_t *d_raw, int64_t *d_filt, void *stream) {
    if (n == 0) return PT_OK;
    PT_CHECK(d_rows && d_row_of && d_truth && d_part_off && d_raw && d_filt && ent_total > 0, PT_EINVAL,
             "pt_rank_rows: null argument");
    PT_HIP(pt::launch_rank_rows(d_rows, ent_total, d_row_of, d_truth, d_repl, d_part_off, d_part, n, d_raw, d_filt,
                                (hipStream_t)stream));
    return PT_OK;
}

extern "C" int pt_rank_types(const float *d_rows, int64_t ent_total, const int64_t *d_row_of, const int64_t *d_truth,
                             const float *d_repl, const int64_t *d_rel, const int64_t *d_type_lef,
                             const int64_t *d_type_rig, const int64_t *d_types, const int64_t *d_part_off,
                             const int64_t *d_part, int64_t n, int64_t *d_raw, int64_t *d_filt, void *stream) {
    if (n == 0) return PT_OK;
    PT_CHECK(d_rows && d_row_of && d_truth && d_rel && d_type_lef && d_type_rig && d_types && d_part_off && d_raw &&
                 d_filt && ent_total > 0,
             PT_EINVAL, "pt_rank_types: null argument");
    PT_HIP(pt::launch_rank_types(d_rows, ent_total, d_row_of, d_truth, d_repl, d_rel, d_type_lef, d_type_rig, d_types,
                                 d_part_off, d_part, n, d_raw, d_filt, (hipStream_t)stream));
    return PT_OK;
}

// ======================================================================== Base.so surface ========
// One process-global context with the reference's semantics (Setting.h / Random.h / Reader.h /
// UniverseSetting.h / Test.h / Valid.h globals). Sampling, training and scoring run on the GPU.
namespace {

struct TestAcc {   // the reference's float accumulators (Test.h:14-21)
    float l_filter_tot = 0, l3_filter_tot = 0, l1_filter_tot = 0, l_filter_rank = 0, l_filter_reci = 0;
    float r_filter_tot = 0, r3_filter_tot = 0, r1_filter_tot = 0, r_filter_rank = 0, r_filter_reci = 0;
    float l_tot = 0, l3_tot = 0, l1_tot = 0, l_rank = 0, l_reci = 0;
    float r_tot = 0, r3_tot = 0, r1_tot = 0, r_rank = 0, r_reci = 0;
};

struct Legacy {
    std::mutex mu;
    std::string in_path = "../data/FB15K/";
    int64_t threads = 1, bern = 0, seed = 0;
    pt::GlibcRand rng{1};
    std::vector<uint64_t> states;
    std::unique_ptr<pt::Graph> train;        // importTrainFiles
    std::string train_path;
    bool train_header = false;               // record format train was read with
    int import_rc = PT_OK;                   // status of the last importTrainFiles / importTestFiles
    std::unique_ptr<pt::Universe> uni;       // getParallelUniverse
    bool swapped = false;
    pt_sampler sampler;                      // device states; g follows the active graph
    bool sampler_ready = false;
    // device batch buffers for the host-pointer sampling()
    int64_t *dbuf = nullptr;
    size_t dbuf_cap = 0;
    // test / valid data
    bool load_all = false;
    int64_t ent_total = 0, rel_total = 0, test_total = 0, valid_total = 0, triple_total = 0, train_lines = 0;
    std::vector<pt::Triple> test, valid;
    pt_known *known = nullptr;
    int64_t last_head = 0, last_tail = 0, last_vhead = 0, last_vtail = 0;
    TestAcc acc, acc_tc;                     // unconstrained / type-constrained accumulators
    float mrr = 0, mr = 0, hit10 = 0, hit3 = 0, hit1 = 0;
    float mrr_tc = 0, mr_tc = 0, hit10_tc = 0, hit3_tc = 0, hit1_tc = 0;
    float l_valid = 0, r_valid = 0, valid_hit10 = 0;
    // importTypeFiles (Reader.h:344-396): per relation [lef, rig) into the sorted head / tail type lists
    bool types_loaded = false;
    std::vector<int64_t> type_lef[2], type_rig[2], type_list[2];

    pt::Graph *active() { return swapped && uni ? &uni->g : train.get(); }
    int64_t E() { pt::Graph *g = active(); return g ? g->ent_total : ent_total; }
};

Legacy &L() {
    static Legacy *l = new Legacy();   // never destroyed: device frees at exit are unsafe
    return *l;
}

void legacy_err(int rc) {
    if (rc) fprintf(stderr, "%s\n", pt_last_error());
}

int legacy_sync_sampler(Legacy &l) {
    if (!l.sampler_ready) {
        int rc = sampler_init(&l.sampler, nullptr, 64, nullptr);
        if (rc) return rc;
        l.sampler.threads = std::max<int64_t>(1, l.threads);
        l.sampler_ready = true;
    }
    l.sampler.g = l.active();
    return PT_OK;
}

int legacy_push_states(Legacy &l) {
    int rc = legacy_sync_sampler(l);
    if (rc) return rc;
    std::vector<uint64_t> s(64, 0);
    std::copy(l.states.begin(), l.states.end(), s.begin());
    PT_HIP(hipMemcpy(l.sampler.d_states, s.data(), sizeof(uint64_t) * 64, hipMemcpyHostToDevice));
    l.sampler.threads = std::max<int64_t>(1, (int64_t)l.states.size());
    return PT_OK;
}

}  // namespace

extern "C" pt_sampler *pt_legacy_sampler(void) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    if (legacy_sync_sampler(l)) return nullptr;
    return &l.sampler;
}

extern "C" void setInPath(char *path) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    l.in_path = path ? path : "";
    printf("Input Files Path : %s\n", l.in_path.c_str());
}
extern "C" void setOutPath(char *path) { (void)path; }
extern "C" void setWorkThreads(int64_t threads) { L().threads = threads; }
extern "C" int64_t getWorkThreads(void) { return L().threads; }
extern "C" void setBern(int64_t con) { L().bern = con; }
extern "C" void setRandomSeed(int64_t seed) {
    Legacy &l = L();
    l.seed = seed == -1 ? (int64_t)time(nullptr) : seed;
    l.rng.seed_with((uint32_t)l.seed);
}
extern "C" int64_t getRandomSeed(void) { return L().seed; }
extern "C" void randReset(void) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    l.states.assign((size_t)std::max<int64_t>(1, l.threads), 0);
    for (auto &s : l.states) s = (uint64_t)(int64_t)l.rng.next();
    legacy_err(legacy_push_states(l));
}
extern "C" void importTrainFiles(void) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    printf("The toolkit is importing datasets.\n");
    if (l.train && l.train_path == l.in_path && l.train_header == pt::count_header() && !l.swapped) {
        l.import_rc = PT_OK;
        return;   // identical re-import
    }
    auto g = std::make_unique<pt::Graph>();
    int rc = pt::load_graph(l.in_path, *g);
    l.import_rc = rc;
    if (rc) {
        legacy_err(rc);
        return;
    }
    (void)hipDeviceSynchronize();   // an older graph may still be read by queued kernels
    l.train = std::move(g);
    l.train_path = l.in_path;
    l.train_header = pt::count_header();
    l.ent_total = l.train->ent_total;
    l.rel_total = l.train->rel_total;
    legacy_err(l.train->upload());
    legacy_err(legacy_sync_sampler(l));
    printf("The total of train triples is %ld.\n", (long)l.train->train_total);
}
// The reference's import functions return void and crash on bad input; ours report through this.
extern "C" int pt_legacy_import_status(void) { return L().import_rc; }
extern "C" int64_t getEntityTotal(void) { Legacy &l = L(); return l.active() ? l.active()->ent_total : l.ent_total; }
extern "C" int64_t getRelationTotal(void) { Legacy &l = L(); return l.active() ? l.active()->rel_total : l.rel_total; }
extern "C" int64_t getTrainTotal(void) { Legacy &l = L(); return l.active() ? l.active()->train_total : l.train_lines; }
extern "C" int64_t getTestTotal(void) { return L().test_total; }
extern "C" int64_t getValidTotal(void) { return L().valid_total; }
extern "C" int64_t getTripleTotal(void) { return L().triple_total; }

extern "C" void sampling(int64_t *bh, int64_t *bt, int64_t *br, float *by, int64_t bs, int64_t neg, int64_t neg_rel,
                         int64_t mode, int64_t filter, int64_t p, int64_t val_loss) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    if (val_loss) {   // positives of the validation list (Base.cpp:255-262)
        for (int64_t b = 0; b < bs && b < (int64_t)l.valid.size(); ++b) {
            bh[b] = l.valid[b].h; bt[b] = l.valid[b].t; br[b] = l.valid[b].r; by[b] = 1;
        }
        return;
    }
    if (neg_rel > 0 && p) {   // corrupt_rel's p branch reads a relation-probability table never loaded
        legacy_err(pt::fail(PT_ENOTSUP, "sampling: p = 1 (probability-weighted corrupt_rel) is not supported"));
        return;
    }
    if (!l.active()) {
        legacy_err(pt::fail(PT_ESTATE, "sampling before importTrainFiles"));
        return;
    }
    int rc = legacy_sync_sampler(l);
    if (rc) return legacy_err(rc);
    const int64_t seq = bs * (1 + neg + neg_rel);
    const size_t need = (size_t)seq * 3 * sizeof(int64_t) + (size_t)seq * sizeof(float);
    if (need > l.dbuf_cap) {
        if (l.dbuf) (void)hipFree(l.dbuf);
        l.dbuf = nullptr;
        if (hipMalloc(&l.dbuf, need) != hipSuccess) return legacy_err(pt::fail(PT_ENOMEM, "sampling buffers"));
        l.dbuf_cap = need;
    }
    int64_t *dh = l.dbuf, *dt = dh + seq, *dr = dt + seq;
    float *dy = (float *)(dr + seq);
    rc = pt_sampler_sample_ex(&l.sampler, bs, neg, neg_rel, mode, l.bern, filter, dh, dt, dr, dy, nullptr);
    if (rc) return legacy_err(rc);
    (void)hipMemcpy(bh, dh, sizeof(int64_t) * seq, hipMemcpyDeviceToHost);
    (void)hipMemcpy(bt, dt, sizeof(int64_t) * seq, hipMemcpyDeviceToHost);
    (void)hipMemcpy(br, dr, sizeof(int64_t) * seq, hipMemcpyDeviceToHost);
    (void)hipMemcpy(by, dy, sizeof(float) * seq, hipMemcpyDeviceToHost);
}

// Neighbourhood getters of TrainDataLoader.get_positive_entities / get_negative_entities /
// get_entity_relations (Base.cpp:312-466) over the active graph (the swapped universe after swapHelpers):
// `is_tail` != 0 scans the entity's run of the cmp_tail list (partners = heads), else its run of the
// cmp_head list (partners = tails); positives are the partners under `relation`, negatives those under
// any other relation, in list order.
static const pt::Graph *legacy_graph_or_null(const char *who) {
    const pt::Graph *g = L().active();
    if (!g) pt::fail(PT_ESTATE, std::string(who) + " before importTrainFiles");
    return g;
}
static int64_t legacy_partners(int64_t entity, int64_t relation, int64_t is_tail, bool positive, int64_t *out) {
    const pt::Graph *g = legacy_graph_or_null("entity neighbourhood getter");
    if (!g || entity < 0 || entity >= g->ent_total) return 0;
    const auto &lst = is_tail ? g->tail : g->head;
    const int64_t lo = is_tail ? g->lef_tail[(size_t)entity] : g->lef_head[(size_t)entity];
    const int64_t hi = is_tail ? g->rig_tail[(size_t)entity] : g->rig_head[(size_t)entity];
    int64_t n = 0;
    for (int64_t i = lo; i <= hi; ++i) {
        const pt::Triple &x = lst[(size_t)i];
        if ((x.r == relation) == positive) {
            if (out) out[n] = is_tail ? x.h : x.t;
            ++n;
        }
    }
    return n;
}
extern "C" int64_t getNumOfNegatives(int64_t entity, int64_t relation, int64_t is_tail) {
    return legacy_partners(entity, relation, is_tail, false, nullptr);
}
extern "C" int64_t getNumOfPositives(int64_t entity, int64_t relation, int64_t is_tail) {
    return legacy_partners(entity, relation, is_tail, true, nullptr);
}
extern "C" void getNegativeEntities(int64_t *out, int64_t entity, int64_t relation, int64_t is_tail) {
    legacy_partners(entity, relation, is_tail, false, out);
}
extern "C" void getPositiveEntities(int64_t *out, int64_t entity, int64_t relation, int64_t is_tail) {
    legacy_partners(entity, relation, is_tail, true, out);
}
static int64_t legacy_entity_relations(int64_t entity, int64_t is_tail, int64_t *out) {
    const pt::Graph *g = legacy_graph_or_null("getEntityRelations");
    if (!g || entity < 0 || entity >= g->ent_total) return 0;
    const auto &lst = is_tail ? g->tail : g->head;
    const int64_t lo = is_tail ? g->lef_tail[(size_t)entity] : g->lef_head[(size_t)entity];
    const int64_t hi = is_tail ? g->rig_tail[(size_t)entity] : g->rig_head[(size_t)entity];
    int64_t n = 0, cur = -1;
    for (int64_t i = lo; i <= hi; ++i) {
        if (lst[(size_t)i].r != cur) {
            cur = lst[(size_t)i].r;
            // the reference never advances its output index (Base.cpp:442-466): every distinct relation
            // lands in out[0], so out[0] ends as the last one and the rest of the buffer is untouched
            if (out) out[0] = cur;
            ++n;
        }
    }
    return n;
}
extern "C" int64_t getNumOfEntityRelations(int64_t entity, int64_t is_tail) {
    return legacy_entity_relations(entity, is_tail, nullptr);
}
extern "C" void getEntityRelations(int64_t *out, int64_t entity, int64_t is_tail) {
    legacy_entity_relations(entity, is_tail, out);
}

extern "C" int64_t pt_legacy_bern(void) { return L().bern; }

// the global context's test / valid lists in the reference's ranking order (cmp_rel2, Reader.h:311-312)
extern "C" int64_t pt_legacy_eval_triples(int32_t valid, int64_t *h, int64_t *t, int64_t *r) {
    Legacy &l = L();
    const std::vector<pt::Triple> &v = valid ? l.valid : l.test;
    if (h && t && r)
        for (size_t i = 0; i < v.size(); ++i) { h[i] = v[i].h; t[i] = v[i].t; r[i] = v[i].r; }
    return (int64_t)v.size();
}
extern "C" const pt_known *pt_legacy_known(void) { return L().known; }
extern "C" pt_graph *pt_legacy_graph(void) {
    // the full training graph of importTrainFiles (never the swapped universe): pt_graph wraps pt::Graph
    return reinterpret_cast<pt_graph *>(L().train.get());
}

extern "C" void getParallelUniverse(int64_t tc, float balance) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    if (!l.train) return legacy_err(pt::fail(PT_ESTATE, "getParallelUniverse before importTrainFiles"));
    l.uni = std::make_unique<pt::Universe>();
    pt::build_universe(*l.train, l.rng, tc, balance, *l.uni);
    printf("Universe configured. \n");
}
extern "C" int64_t getEntityTotalUniverse(void) {
    Legacy &l = L();
    if (!l.uni) return 0;
    return l.swapped ? l.train->ent_total : l.uni->g.ent_total;
}
extern "C" int64_t getRelationTotalUniverse(void) {
    Legacy &l = L();
    if (!l.uni) return 0;
    return l.swapped ? l.train->rel_total : l.uni->g.rel_total;
}
extern "C" int64_t getTrainTotalUniverse(void) {
    Legacy &l = L();
    if (!l.uni) return 0;
    return l.swapped ? l.train->train_total : l.uni->g.train_total;
}
extern "C" void getEntityRemapping(int64_t *out) {
    Legacy &l = L();
    if (l.uni) std::copy(l.uni->ent_remap.begin(), l.uni->ent_remap.end(), out);
}
extern "C" void getRelationRemapping(int64_t *out) {
    Legacy &l = L();
    if (l.uni) std::copy(l.uni->rel_remap.begin(), l.uni->rel_remap.end(), out);
}
extern "C" void swapHelpers(void) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    if (!l.uni) return legacy_err(pt::fail(PT_ESTATE, "swapHelpers without a universe"));
    l.swapped = !l.swapped;
    if (l.swapped) legacy_err(l.uni->g.upload());
    legacy_err(legacy_sync_sampler(l));
}
extern "C" void resetUniverse(void) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    l.swapped = false;
    (void)hipDeviceSynchronize();   // queued steps may still read the universe graph
    l.uni.reset();
    legacy_err(legacy_sync_sampler(l));
}

// ----------------------------------------------------------------------- test / valid ----------
// A test / valid / train / triple2id list under the current record format (graph.h record_count).
static bool read_list(const std::string &path, std::vector<pt::Triple> &out) {
    bool ok = true;
    std::string err;
    const int64_t n = pt::record_count(path, &ok, &err);
    if (!ok) return false;
    return pt::read_triples(path, n, out) && (!pt::count_header() || (int64_t)out.size() == n);
}

extern "C" void activateLoadOfAllTriples(int64_t) { L().load_all = true; }

extern "C" void importTestFiles(void) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    bool ok = true;
    l.rel_total = pt::record_count(l.in_path + "relation2id.txt", &ok);
    l.ent_total = pt::record_count(l.in_path + "entity2id.txt", &ok);
    std::vector<pt::Triple> train_all;
    l.import_rc = PT_EIO;
    if (!ok || !read_list(l.in_path + "test2id.txt", l.test) || !read_list(l.in_path + "train2id.txt", train_all) ||
        !read_list(l.in_path + "valid2id.txt", l.valid))
        return legacy_err(pt::fail(PT_EIO, "importTestFiles: missing or malformed test/train/valid file under " +
                                               l.in_path));
    l.test_total = (int64_t)l.test.size();
    l.valid_total = (int64_t)l.valid.size();
    l.train_lines = (int64_t)train_all.size();
    std::vector<pt::Triple> all;
    if (l.load_all) {
        if (!read_list(l.in_path + "triple2id.txt", all))
            return legacy_err(pt::fail(PT_EIO, "importTestFiles: triple2id.txt missing"));
    } else {
        all = l.test;
        all.insert(all.end(), train_all.begin(), train_all.end());
        all.insert(all.end(), l.valid.begin(), l.valid.end());
    }
    l.triple_total = (int64_t)all.size();
    // type lists read for an earlier import belong to that dataset: a type-constrained ranking of this one
    // reads its own type_constrain.txt (importTypeFiles again, or the drop-in Tester's load on first use)
    l.types_loaded = false;
    std::vector<int64_t> h(all.size()), t(all.size()), r(all.size());
    for (size_t i = 0; i < all.size(); ++i) { h[i] = all[i].h; t[i] = all[i].t; r[i] = all[i].r; }
    pt_known *k = nullptr;
    pt_known_create(h.data(), t.data(), r.data(), (int64_t)all.size(), &k);
    if (l.known) pt_known_free(l.known);
    l.known = k;
    l.import_rc = PT_OK;
    std::sort(l.test.begin(), l.test.end(), pt::cmp_rel2);    // Reader.h:311-312
    std::sort(l.valid.begin(), l.valid.end(), pt::cmp_rel2);
    printf("The total of test triples is %ld.\n", (long)l.test_total);
}

namespace pt {
void rank_one(const pt_known &k, int64_t E, int64_t h, int64_t t, int64_t r, int side, const float *con,
              int64_t *raw, int64_t *filt);
bool known_has(const pt_known &k, int64_t h, int64_t t, int64_t r);
}

// ------------------------------------------------------------------ triple classification -------
namespace {
// corrupt_head / corrupt_tail with the known-triple filter (Corrupt.h:9-105, filter_flag true) over the
// training graph's sorted lists on the host: heads = 1 draws a replacement TAIL for (key = h, r) from
// trainHead, heads = 0 a replacement HEAD for (key = t, r) from trainTail. An entity without training
// triples makes the reference read trainHead[-1] (its ll is -1): that is the calloc block's header,
// larger than any entity id, so `tmp < trainHead[ll].t` holds and the draw is returned as is - emulated
// by reading index -1 as "larger than every id" (index n, never reached by a non-empty list, likewise).
int64_t host_corrupt(const pt::Graph &g, bool heads, int64_t key, int64_t r, uint64_t &state) {
    const std::vector<pt::Triple> &L = heads ? g.head : g.tail;
    const std::vector<int64_t> &lef = heads ? g.lef_head : g.lef_tail, &rig = heads ? g.rig_head : g.rig_tail;
    const int64_t n = (int64_t)L.size();
    auto val = [&](int64_t k) -> int64_t {
        if (k < 0 || k >= n) return INT64_MAX / 4;
        return heads ? L[(size_t)k].t : L[(size_t)k].h;
    };
    int64_t lo = lef[(size_t)key] - 1, hi = rig[(size_t)key], mid;
    while (lo + 1 < hi) {
        mid = (lo + hi) >> 1;
        if (L[(size_t)mid].r >= r) hi = mid; else lo = mid;
    }
    const int64_t ll = hi;
    lo = lef[(size_t)key];
    hi = rig[(size_t)key] + 1;
    while (lo + 1 < hi) {
        mid = (lo + hi) >> 1;
        if (L[(size_t)mid].r <= r) lo = mid; else hi = mid;
    }
    const int64_t rr = lo;
    state = state * 25214903917ULL + 11ULL;   // randd (Random.h:18-22)
    const int64_t tmp = (int64_t)(state % (uint64_t)(g.ent_total - (rr - ll + 1)));
    if (tmp < val(ll)) return tmp;
    if (tmp > val(rr) - rr + ll - 1) return tmp + rr - ll + 1;
    lo = ll;
    hi = rr + 1;
    while (lo + 1 < hi) {
        mid = (lo + hi) >> 1;
        if (val(mid) - mid + ll - 1 < tmp) lo = mid; else hi = mid;
    }
    return tmp + lo - ll + 1;
}
}  // namespace

// getTestBatch (Test.h:576-599): the test triples and one negative each - a coin from sampler thread 0
// (randd(0) % 1000 < 500) picks corrupt_head(0, h, r) (new tail) or corrupt_tail(0, t, r) (new head).
// The stream is the process-global sampler's thread 0 (device-resident here: read, advanced, written
// back), so the negatives continue the same random sequence as in the reference.
extern "C" void getTestBatch(int64_t *ph, int64_t *pt_, int64_t *pr, int64_t *nh, int64_t *nt, int64_t *nr) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    pt::Graph *g = l.train.get();
    if (!g || g->ent_total < 2) {
        legacy_err(pt::fail(PT_ESTATE, "getTestBatch: importTrainFiles() first"));
        return;
    }
    uint64_t s0 = l.states.empty() ? 0 : l.states[0];
    if (l.sampler_ready && hipMemcpy(&s0, l.sampler.d_states, sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) {
        legacy_err(pt::fail(PT_EHIP, "getTestBatch: reading the sampler state failed"));
        return;
    }
    for (size_t i = 0; i < l.test.size(); ++i) {
        const pt::Triple &q = l.test[i];
        pt::Triple neg = q;
        s0 = s0 * 25214903917ULL + 11ULL;
        if ((int64_t)(s0 % 1000ULL) < 500) neg.t = host_corrupt(*g, true, q.h, q.r, s0);
        else neg.h = host_corrupt(*g, false, q.t, q.r, s0);
        ph[i] = q.h; pt_[i] = q.t; pr[i] = q.r;
        nh[i] = neg.h; nt[i] = neg.t; nr[i] = neg.r;
    }
    if (!l.states.empty()) l.states[0] = s0;
    if (l.sampler_ready &&
        hipMemcpy(l.sampler.d_states, &s0, sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess)
        legacy_err(pt::fail(PT_EHIP, "getTestBatch: writing the sampler state failed"));
}

extern "C" void initTest(void) {
    Legacy &l = L();
    l.last_head = l.last_tail = 0;
    l.acc = TestAcc{};
    l.acc_tc = TestAcc{};
}

static void fill_batch(const pt::Triple &q, int64_t E, int side, int64_t *ph, int64_t *pt_, int64_t *pr) {
    ph[0] = q.h; pt_[0] = q.t; pr[0] = q.r;
    const int64_t truth = side == 0 ? q.h : q.t;
    for (int64_t i = 1; i < E; ++i) {
        const int64_t c = i - 1 < truth ? i - 1 : i;
        ph[i] = side == 0 ? c : q.h;
        pt_[i] = side == 0 ? q.t : c;
        pr[i] = q.r;
    }
}

extern "C" void getHeadBatch(int64_t *ph, int64_t *pt_, int64_t *pr) {
    Legacy &l = L();
    fill_batch(l.test[(size_t)l.last_head++], l.ent_total, 0, ph, pt_, pr);
}
extern "C" void getTailBatch(int64_t *ph, int64_t *pt_, int64_t *pr) {
    Legacy &l = L();
    fill_batch(l.test[(size_t)l.last_tail++], l.ent_total, 1, ph, pt_, pr);
}

static void accumulate(TestAcc &a, int side, int64_t raw, int64_t filt) {
    float &ft = side == 0 ? a.l_filter_tot : a.r_filter_tot, &f3 = side == 0 ? a.l3_filter_tot : a.r3_filter_tot,
          &f1 = side == 0 ? a.l1_filter_tot : a.r1_filter_tot, &fr = side == 0 ? a.l_filter_rank : a.r_filter_rank,
          &fi = side == 0 ? a.l_filter_reci : a.r_filter_reci;
    float &rt = side == 0 ? a.l_tot : a.r_tot, &r3 = side == 0 ? a.l3_tot : a.r3_tot,
          &r1 = side == 0 ? a.l1_tot : a.r1_tot, &rr = side == 0 ? a.l_rank : a.r_rank,
          &ri = side == 0 ? a.l_reci : a.r_reci;
    if (filt < 10) ft += 1;
    if (raw < 10) rt += 1;
    if (filt < 3) f3 += 1;
    if (raw < 3) r3 += 1;
    if (filt < 1) f1 += 1;
    if (raw < 1) r1 += 1;
    fr += (float)(filt + 1);
    rr += (float)(1 + raw);
    fi = (float)((double)fi + 1.0 / (double)(filt + 1));
    ri = (float)((double)ri + 1.0 / (double)(raw + 1));
}

// importTypeFiles (Reader.h:352-396): `type_constrain.txt` in the input folder - a count, then for each of
// relationTotal relations a line of head types and a line of tail types, `r n e_1 .. e_n`; every list is
// sorted in place. (The reference's Python never calls it; testHead/testTail with type_constrain read
// these arrays.)
extern "C" void importTypeFiles(void) {
    Legacy &l = L();
    std::lock_guard<std::mutex> lk(l.mu);
    const std::string path = l.in_path + "type_constrain.txt";
    FILE *f = fopen(path.c_str(), "r");
    if (!f) return legacy_err(pt::fail(PT_EIO, "importTypeFiles: cannot open " + path));
    const int64_t R = l.rel_total;
    for (int s = 0; s < 2; ++s) {
        l.type_lef[s].assign((size_t)R, 0);
        l.type_rig[s].assign((size_t)R, 0);
        l.type_list[s].clear();
    }
    long tmp = 0;
    bool ok = fscanf(f, "%ld", &tmp) == 1;
    for (int64_t i = 0; ok && i < R; ++i) {
        for (int s = 0; s < 2 && ok; ++s) {
            long rel = 0, tot = 0;
            ok = fscanf(f, "%ld %ld", &rel, &tot) == 2 && rel >= 0 && rel < R && tot >= 0;
            if (!ok) break;
            std::vector<int64_t> &v = l.type_list[s];
            l.type_lef[s][(size_t)rel] = (int64_t)v.size();
            for (long j = 0; j < tot && ok; ++j) {
                long e = 0;
                ok = fscanf(f, "%ld", &e) == 1;
                v.push_back(e);
            }
            l.type_rig[s][(size_t)rel] = (int64_t)v.size();
            std::sort(v.begin() + l.type_lef[s][(size_t)rel], v.end());
        }
    }
    fclose(f);
    l.types_loaded = ok;
    if (!ok) legacy_err(pt::fail(PT_EIO, "importTypeFiles: malformed " + path));
}

// Type-constrained counts of one query (Test.h:168-178 / :288-298). The reference walks candidate
// POSITIONS j = 1..E-1 and matches j against the relation's sorted type list as an ENTITY id, so the
// score it compares for type entity j is con[j] (the candidate at position j) and the filter asks
// _find about entity j; nothing is counted when con[0] == inf. Restated as is.
static void rank_constrained(const Legacy &l, const pt::Triple &q, int side, const float *con, int64_t *raw,
                             int64_t *filt) {
    int64_t s = 0, fs = 0;
    const float minimal = con[0];
    if (minimal != INFINITY) {
        const std::vector<int64_t> &v = l.type_list[side];
        const int64_t lo = l.type_lef[side][(size_t)q.r], hi = l.type_rig[side][(size_t)q.r];
        for (int64_t k = lo; k < hi; ++k) {
            const int64_t j = v[(size_t)k];
            if (j < 1 || j >= l.ent_total || (k > lo && v[(size_t)k - 1] == j)) continue;
            if (con[j] < minimal) {
                ++s;
                if (!(side == 0 ? pt::known_has(*l.known, j, q.t, q.r) : pt::known_has(*l.known, q.h, j, q.r))) ++fs;
            }
        }
    }
    *raw = s;
    *filt = fs;
}

static void test_one(float *con, int64_t idx, int64_t type_constrain, int side) {
    Legacy &l = L();
    const pt::Triple &q = l.test[(size_t)idx];
    int64_t raw, filt;
    pt::rank_one(*l.known, l.ent_total, q.h, q.t, q.r, side, con, &raw, &filt);
    accumulate(l.acc, side, raw, filt);
    if (type_constrain) {
        if (!l.types_loaded) {
            legacy_err(pt::fail(PT_ESTATE, "type_constrain needs importTypeFiles() first (the reference reads "
                                           "unallocated type arrays, Test.h:127-130)"));
            return;
        }
        rank_constrained(l, q, side, con, &raw, &filt);
        accumulate(l.acc_tc, side, raw, filt);
    }
}
extern "C" void testHead(float *con, int64_t idx, int64_t type_constrain) { test_one(con, idx, type_constrain, 0); }
extern "C" void testTail(float *con, int64_t idx, int64_t type_constrain) { test_one(con, idx, type_constrain, 1); }

// test_link_prediction's averaging (Test.h:408-454, constrained block :456-502)
static void finish_acc(TestAcc &a, float n, float out[5]) {
    a.l_rank /= n; a.r_rank /= n; a.l_reci /= n; a.r_reci /= n;
    a.l_tot /= n; a.l3_tot /= n; a.l1_tot /= n; a.r_tot /= n; a.r3_tot /= n; a.r1_tot /= n;
    a.l_filter_rank /= n; a.r_filter_rank /= n; a.l_filter_reci /= n; a.r_filter_reci /= n;
    a.l_filter_tot /= n; a.l3_filter_tot /= n; a.l1_filter_tot /= n;
    a.r_filter_tot /= n; a.r3_filter_tot /= n; a.r1_filter_tot /= n;
    out[0] = (a.l_filter_reci + a.r_filter_reci) / 2;
    out[1] = (a.l_filter_rank + a.r_filter_rank) / 2;
    out[2] = (a.l_filter_tot + a.r_filter_tot) / 2;
    out[3] = (a.l3_filter_tot + a.r3_filter_tot) / 2;
    out[4] = (a.l1_filter_tot + a.r1_filter_tot) / 2;
}

extern "C" void test_link_prediction(int64_t type_constrain) {
    Legacy &l = L();
    if (type_constrain) {
        float m[5];
        finish_acc(l.acc_tc, (float)l.test_total, m);
        l.mrr_tc = m[0]; l.mr_tc = m[1]; l.hit10_tc = m[2]; l.hit3_tc = m[3]; l.hit1_tc = m[4];
        printf("type constraint results:\n");
        printf("averaged(filter):\t %f \t %f \t %f \t %f \t %f \n", m[0], m[1], m[2], m[3], m[4]);
    }
    TestAcc &a = l.acc;
    float m[5];
    finish_acc(a, (float)l.test_total, m);
    printf("metric:\t\t\t MRR \t\t MR \t\t hit@10 \t hit@3  \t hit@1 \n");
    printf("averaged(raw):\t\t %f \t %f \t %f \t %f \t %f \n", (a.l_reci + a.r_reci) / 2, (a.l_rank + a.r_rank) / 2,
           (a.l_tot + a.r_tot) / 2, (a.l3_tot + a.r3_tot) / 2, (a.l1_tot + a.r1_tot) / 2);
    l.mrr = m[0]; l.mr = m[1]; l.hit10 = m[2]; l.hit3 = m[3]; l.hit1 = m[4];
    printf("averaged(filter):\t %f \t %f \t %f \t %f \t %f \n", l.mrr, l.mr, l.hit10, l.hit3, l.hit1);
}
extern "C" float getTestLinkMRR(int64_t tc) { return tc ? L().mrr_tc : L().mrr; }
extern "C" float getTestLinkMR(int64_t tc) { return tc ? L().mr_tc : L().mr; }
extern "C" float getTestLinkHit10(int64_t tc) { return tc ? L().hit10_tc : L().hit10; }
extern "C" float getTestLinkHit3(int64_t tc) { return tc ? L().hit3_tc : L().hit3; }
extern "C" float getTestLinkHit1(int64_t tc) { return tc ? L().hit1_tc : L().hit1; }

// the loaded type lists for the GPU ranking: side 0 heads, 1 tails; lef/rig per relation (relTotal
// entries each) and the lists; returns the list length (-1 before importTypeFiles). NULL outputs skip.
extern "C" int64_t pt_legacy_types(int32_t side, int64_t *lef, int64_t *rig, int64_t *list) {
    Legacy &l = L();
    if (!l.types_loaded || (side != 0 && side != 1)) return -1;
    const auto &lv = l.type_lef[side], &rv = l.type_rig[side], &tv = l.type_list[side];
    if (lef) std::copy(lv.begin(), lv.end(), lef);
    if (rig) std::copy(rv.begin(), rv.end(), rig);
    if (list) std::copy(tv.begin(), tv.end(), list);
    return (int64_t)tv.size();
}

extern "C" void validInit(void) {
    Legacy &l = L();
    l.last_vhead = l.last_vtail = 0;
    l.l_valid = l.r_valid = 0;
}
extern "C" void getValidHeadBatch(int64_t *ph, int64_t *pt_, int64_t *pr) {
    Legacy &l = L();
    fill_batch(l.valid[(size_t)l.last_vhead++], l.ent_total, 0, ph, pt_, pr);
}
extern "C" void getValidTailBatch(int64_t *ph, int64_t *pt_, int64_t *pr) {
    Legacy &l = L();
    fill_batch(l.valid[(size_t)l.last_vtail++], l.ent_total, 1, ph, pt_, pr);
}
extern "C" void validHead(float *con, int64_t idx) {
    Legacy &l = L();
    const pt::Triple &q = l.valid[(size_t)idx];
    int64_t raw, filt;
    pt::rank_one(*l.known, l.ent_total, q.h, q.t, q.r, 0, con, &raw, &filt);
    if (filt < 10) l.l_valid += 1;
}
extern "C" void validTail(float *con, int64_t idx) {
    Legacy &l = L();
    const pt::Triple &q = l.valid[(size_t)idx];
    int64_t raw, filt;
    pt::rank_one(*l.known, l.ent_total, q.h, q.t, q.r, 1, con, &raw, &filt);
    if (filt < 10) l.r_valid += 1;
}
extern "C" float getValidHit10(void) {
    Legacy &l = L();
    l.l_valid /= (float)l.valid_total;
    l.r_valid /= (float)l.valid_total;
    l.valid_hit10 = (l.l_valid + l.r_valid) / 2;
    return l.valid_hit10;
}
