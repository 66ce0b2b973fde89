/*
 * putranse.h — C-ABI of libputranse_hip.so, the MI355X-native PuTransE / TransE / TransH hot path.
 *
 * Two surfaces, both plain C (pointers + sizes, no torch types):
 *
 *  A. Reentrant GPU entry points (pt_*): explicit handles, device pointers owned by the caller
 *     (torch tensors), a hipStream_t passed as void*, int status returns (0 = ok, else a PT_E* code;
 *     pt_last_error() gives the message). Nothing here calls exit().
 *
 *  B. The reference's Base.so symbols for this path (same names, argument meaning and global-state
 *     semantics as openke/base/Base.cpp + headers), so a ctypes caller written against Base.so
 *     (TrainDataLoader.py:30-101, TestDataLoader.py:220-266, Tester.py:20-36) binds unchanged.
 *     They run on one process-global default context; batch construction, training and scoring
 *     still execute on the GPU (host buffers are copied over PCIe).
 *
 * Integer ids are int64 (the reference's INT = long, Setting.h:3), reals float32 (REAL, Setting.h:4).
 */
#ifndef PUTRANSE_H
#define PUTRANSE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status ------------------ */
enum {
    PT_OK = 0,
    PT_EINVAL = 1,   /* bad argument / shape */
    PT_EIO = 2,      /* dataset file missing or malformed */
    PT_ENOMEM = 3,   /* host or device allocation failed */
    PT_EHIP = 4,     /* a HIP runtime call failed */
    PT_ESTATE = 5,   /* call out of order (e.g. no dataset imported) */
    PT_ENOTSUP = 6   /* configuration the kernels do not implement */
};
const char *pt_last_error(void);
int pt_version(void);                /* ABI version, bumped on incompatible change */

/* ------------------------------------------------------------------ graphs ------------------ */
/* A training graph: deduplicated triples in cmp_head order plus the helper indices the sampler
 * needs (replaces importTrainFiles + loadHelpers, Reader.h:58-234). */
typedef struct pt_graph pt_graph;
int pt_graph_load(const char *in_path, pt_graph **out);   /* h t r files; line-counted unless count-header */
/* Record format of every *2id.txt reader in this library (pt_graph_load, importTrainFiles,
 * importTestFiles), process-global like setInPath. 0 (default): the reference's contract, the line count
 * is the record count (Reader.h:176-196, Utilities.h:47-57). 1: the first line holds the record count,
 * the upstream OpenKE format of the FB15K237 / WN18RR / FB13 / WN11 / NELL folders (the fscanf this fork
 * commented out at Reader.h:178,185,191); a malformed or short file is then an error. */
int pt_set_count_header(int on);
int pt_get_count_header(void);
int pt_graph_free(pt_graph *g);
int64_t pt_graph_ent_total(const pt_graph *g);
int64_t pt_graph_rel_total(const pt_graph *g);
int64_t pt_graph_train_total(const pt_graph *g);
/* copies the cmp_head-ordered training triples to host arrays of length train_total */
int pt_graph_triples(const pt_graph *g, int64_t *h, int64_t *t, int64_t *r);

/* ------------------------------------------------------------------ sampler ----------------- */
/* Device sampler bound to a graph: reproduces sampling()/getBatch() (Base.cpp:185-310) bit for bit
 * for a given (seed states, threads) — `threads` only names the RNG-stream partition emulated. */
typedef struct pt_sampler pt_sampler;
int pt_sampler_create(pt_graph *g, int64_t threads, const uint64_t *seeds, pt_sampler **out);
int pt_sampler_free(pt_sampler *s);
/* re-seed the per-thread LCG streams (randReset, Random.h:10-15) */
int pt_sampler_set_seeds(pt_sampler *s, const uint64_t *seeds);
int pt_sampler_get_seeds(pt_sampler *s, uint64_t *seeds);       /* current states (host copy) */
/* one sampling() call into DEVICE arrays of length bs*(1+neg); advances the streams */
int pt_sampler_sample(pt_sampler *s, int64_t bs, int64_t neg, int64_t bern, int64_t filter, int64_t *d_h,
                      int64_t *d_t, int64_t *d_r, float *d_y, void *stream);
/* sampling() with its mode and relation corruptions (Base.cpp:185-264; replaces the mode / negRelRate
 * arguments of Base.cpp:266-279 bound at TrainDataLoader.py:33-45 and used by sampling_head /
 * sampling_tail / cross_sampling, TrainDataLoader.py:198-246): mode 0 normal, -1 head_batch (heads
 * replaced by corrupt_tail), 1 tail_batch (tails replaced by corrupt_head); neg_rel relation corruptions
 * per positive (corrupt_rel, p = false). DEVICE arrays of length bs*(1+neg+neg_rel). PT_EINVAL when
 * neg_rel > 0 and some (h,t) pair holds every relation (the reference divides by zero there). */
int pt_sampler_sample_ex(pt_sampler *s, int64_t bs, int64_t neg, int64_t neg_rel, int64_t mode, int64_t bern,
                         int64_t filter, int64_t *d_h, int64_t *d_t, int64_t *d_r, float *d_y, void *stream);

/* ------------------------------------------------------------------ training ---------------- */
enum { PT_TRANSE = 0, PT_TRANSH = 1 };
enum { PT_SGD = 0, PT_ADAGRAD = 1 };

typedef struct {
    int32_t model;        /* PT_TRANSE | PT_TRANSH */
    int32_t p_norm;       /* 1 or 2  (TransE.py:46-60) */
    int32_t norm_flag;    /* F.normalize of h, r, t before scoring */
    int32_t opt;          /* PT_SGD | PT_ADAGRAD (Trainer.py:62-88; eps 1e-10, lr_decay 0) */
    float lr;
    float margin;         /* MarginLoss margin (MarginLoss.py:24-28) */
    int64_t ent_total, rel_total, dim;
    float *ent, *rel, *normv;              /* device tables [rows][dim], row-major fp32 */
    float *ent_acc, *rel_acc, *norm_acc;   /* Adagrad state_sum (NULL for SGD) */
} pt_model_desc;

/* Workspace for minibatch-synchronous steps on one model (gradient rows, touched-row flags). */
typedef struct pt_trainer pt_trainer;
int pt_trainer_create(const pt_model_desc *m, pt_trainer **out);
int pt_trainer_free(pt_trainer *t);
int pt_trainer_update_desc(pt_trainer *t, const pt_model_desc *m);   /* new lr/margin/pointers */
/* One training step = Trainer.train_one_step (Trainer.py:44-56): NegativeSampling + MarginLoss
 * forward, analytic backward, sparse optimizer update.  Batch either sampled in-kernel from
 * `sampler` (batch_h == NULL) or read from device arrays of length bs*(1+neg) in the reference
 * layout (negative k of positive i at (k+1)*bs+i).  Adds the step's loss to *d_loss (device). */
int pt_trainer_step(pt_trainer *t, pt_sampler *sampler, int64_t bs, int64_t neg, int64_t bern, int64_t filter,
                    const int64_t *d_batch_h, const int64_t *d_batch_t, const int64_t *d_batch_r, float *d_loss,
                    void *stream);
/* `steps` consecutive in-kernel-sampled steps (one epoch = nbatches steps), launch-overhead-free
 * (captured once into a hipGraph per shape and replayed). d_losses[s] receives step s's loss. */
int pt_trainer_run(pt_trainer *t, pt_sampler *sampler, int64_t bs, int64_t neg, int64_t bern, int64_t filter,
                   int64_t steps, float *d_losses, void *stream);

/* Sampling path of the trainer's in-kernel-sampled chunks (neg >= 4): path = PT_PATH_FUSED / PT_PATH_PART /
 * PT_PATH_TWO_PASS (where its LDS plan fits) or -1 (automatic: fused for chunks of >= 96 steps, else the split
 * sampler); parts = workgroups per call of the split sampler (0 = automatic, ceil(512 / calls)). Every path
 * draws the same batches (bit-exact); this selects only how. */
int pt_trainer_set_sampling(pt_trainer *t, int32_t path, int64_t parts);
/* Split-sampler chunks sampled in two launches (same batches, bit-exact): the first `head` steps ahead of the
 * first step, the rest on the trainer's side stream alongside the first steps' training. head = 0 or -1 (the
 * default): one launch (measured faster); a chunk of <= head steps is sampled in one launch. */
int pt_trainer_set_sample_split(pt_trainer *t, int64_t head);
/* Reference-order (deterministic) mode of a trainer: every later pt_trainer_step / pt_trainer_run sums each
 * table row's gradient in slot order, lookup by lookup (batch_h, batch_t, batch_r; norm_vector(batch_r)),
 * as torch's embedding_dense_backward + AccumulateGrad do for Trainer.train_one_step (Trainer.py:44-56),
 * with sequential dot products / norms and IEEE division and square root. Results are bit-identical run to
 * run (and to the CPU restatement oracle/oracle.c); the default fast path sums the same contributions in
 * arrival order (float atomics) and is faster. on = 0 returns to the fast path. */
int pt_trainer_set_deterministic(pt_trainer *t, int32_t on);
int pt_trainer_get_deterministic(const pt_trainer *t);

/* Measurement hook: `steps` in-kernel-sampled steps launched one by one (no graph) with an event pair
 * around every launch on `stream`. ms4[k] = total duration of kernel kind k divided by `steps`:
 * 0 batch sampling (k_sample_csr, large-neg path only, one launch per chunk of steps), 1 bucket scan
 * (k_scan_counts, idem), 2 fused forward/backward (k_step_csr / k_step_sampled), 3 sparse optimizer
 * (k_apply_buf / k_apply). On the large-neg path kinds 2 and 3 are then re-timed back to back (one
 * event pair per loop of `steps` launches on the last sampled batch; tables, optimizer state and
 * gradient rows restored), as the captured epoch runs them. Synchronizes the stream. */
int pt_trainer_run_timed(pt_trainer *t, pt_sampler *sampler, int64_t bs, int64_t neg, int64_t bern, int64_t filter,
                         int64_t steps, float *d_losses, float *ms4, void *stream);
/* Sampling path the last enqueued in-kernel-sampled chunk took (for reports): kinds 0/1 of ms4 are then
 * PT_PATH_FUSED: k_sample_sort + k_advance; PT_PATH_PART: k_sample_part + k_resolve; PT_PATH_TWO_PASS:
 * k_sample_csr + k_scan_counts; PT_PATH_SAMPLED: none (small neg: the step kernel samples). -1 before any. */
enum { PT_PATH_TWO_PASS = 0, PT_PATH_FUSED = 1, PT_PATH_PART = 2, PT_PATH_SAMPLED = 3 };
int pt_trainer_last_path(const pt_trainer *t);
/* The large-neg TransE step as ONE launch that also updates the table rows (step_apply.hip: each row
 * updated inside the step by the wave delivering its last gradient contribution, same operations and
 * order as the separate apply pass), for float4 rows of 33-256 chunks (dim 132-1024, dim % 4 == 0);
 * on = 0 keeps the step + apply pair. Default off (measured slower at C2: DESIGN.md section 4). Results
 * equal the pair's up to float-atomic order. */
int pt_trainer_set_step_apply(pt_trainer *t, int32_t on);
/* slot-scale mode (opt-in; TransE float4 rows on the counting-sort path): the step stores per (positive, negative)
 * slot a record (positive, side, one scalar) and per positive its three normalized rows instead of the corrupted
 * entity's gradient row, and the apply pass re-forms each slot's row from them and the entity's own row
 * (CsrWork::slot_scale). pt_trainer_slot_scale: 1 when the current workspace is carved for it. */
int pt_trainer_set_slot_scale(pt_trainer *t, int32_t on);
int pt_trainer_slot_scale(const pt_trainer *t);
/* whether the last enqueued in-kernel-sampled steps took the fused step + apply (ms4[2] of
 * pt_trainer_run_timed is then that kernel, ms4[3] the chunks' loss reduction) */
int pt_trainer_step_apply(const pt_trainer *t);
/* Sample `calls` consecutive steps into the counting-sort batch layout the large-neg step kernels read,
 * by path `path` (PT_PATH_FUSED / PT_PATH_PART / PT_PATH_TWO_PASS, or -1 = the automatic choice), advance
 * the sampler streams, and copy the batches to HOST arrays (synchronizes): h_pos [calls][bs][3] (h, r, t
 * of each positive), h_neg [calls][bs*neg] (corrupted entity << 1 | 1 when the tail was replaced, slot
 * b*neg + k = negative k of positive b, Base.cpp:216-232), h_dst [calls][bs*neg] (the slot's row in its
 * entity's bucket: h_start[e] <= dst < h_start[e+1]), h_start [calls][ent_total + 1]. */
int pt_trainer_sample_csr(pt_trainer *t, pt_sampler *sampler, int64_t bs, int64_t neg, int64_t bern, int64_t filter,
                          int64_t calls, int32_t path, int32_t *h_pos, int32_t *h_neg, int32_t *h_dst,
                          int32_t *h_start, void *stream);

/* ------------------------------------------------------------------ scoring ------------------ */
/* scores = ||h + r - t||_p as model.predict computes them (TransE.py:46-74, TransH.py:52-93):
 * mode 0 normal (all three arrays length n), 1 head_batch (d_h length n, t and r length 1),
 * 2 tail_batch (d_t length n, h and r length 1). */
int pt_score(const pt_model_desc *m, int32_t mode, const int64_t *d_h, const int64_t *d_t, const int64_t *d_r,
             int64_t n, float *d_out, void *stream);

/* Link-prediction candidate scores: row q = query q's candidates in getHeadBatch/getTailBatch order
 * ([truth, 0..E-1 without truth], Test.h:37-107). side 0: head prediction (scores (e, r, t), association
 * e + (r - t)); side 1: tail prediction ((h + r) - e). d_out is [nq][ent_total]; nq <= 65535. */
int pt_score_queries(const pt_model_desc *m, int32_t side, const int64_t *d_qh, const int64_t *d_qt,
                     const int64_t *d_qr, int64_t nq, float *d_out, void *stream);
/* the same scores in global entity order (column e = entity e), the layout pt_rank_rows ranks */
int pt_score_rows(const pt_model_desc *m, int32_t side, const int64_t *d_qh, const int64_t *d_qt,
                  const int64_t *d_qr, int64_t nq, float *d_out, void *stream);
/* Metrics from per-query ranks with the reference's float accumulation (Test.h:213-223, :398-454):
 * metrics[0..4] = filtered {MRR, MR, Hits@10, Hits@3, Hits@1}, metrics[5..9] = the raw ones. */
int pt_lp_metrics(const int64_t *rank_head, const int64_t *frank_head, const int64_t *rank_tail,
                  const int64_t *frank_tail, int64_t n, float *metrics);

/* ------------------------------------------------------------------ universes --------------- */
/* Universe construction (getParallelUniverse, UniverseConstructor.h:327-397) with private glibc-
 * compatible RNG state seeded like setRandomSeed(seed)+randReset() (Random.h:10-15, :37-45), so
 * universe k is a pure function of (graph, seed0+k, tc, balance) and many can be built in parallel. */
typedef struct pt_universe pt_universe;
int pt_universe_build(const pt_graph *g, int64_t seed, int64_t threads, int64_t triple_constraint,
                      float balance, pt_universe **out);
int pt_universe_free(pt_universe *u);
/* build n universes on host threads: seeds[i], tcs[i], balances[i] -> out[i] */
int pt_universe_build_many(const pt_graph *g, int64_t n, const int64_t *seeds, int64_t threads,
                           const int64_t *tcs, const float *balances, int64_t n_workers, pt_universe **out);
int64_t pt_universe_ent_total(const pt_universe *u);
int64_t pt_universe_rel_total(const pt_universe *u);
int64_t pt_universe_train_total(const pt_universe *u);
int pt_universe_remaps(const pt_universe *u, int64_t *ent_remap, int64_t *rel_remap);   /* local -> global */
pt_graph *pt_universe_graph(pt_universe *u);      /* the universe's local training graph */
int pt_universe_seeds(const pt_universe *u, uint64_t *seeds);   /* LCG states after randReset */

/* Train many universes concurrently: one persistent workgroup per universe runs all its epochs x
 * nbatches minibatch-synchronous steps (Parallel_Universe_Config.train_embedding_space + Trainer.run,
 * Parallel_Universe_Config.py:228-258, Trainer.py:90-104), universes of different dims on separate
 * streams. Tables / accumulators are the caller's device buffers (updated in place). */
typedef struct {
    const pt_graph *graph;      /* universe-local training graph (from pt_universe_graph) */
    const uint64_t *seeds;      /* host: `threads` LCG states (pt_universe_seeds) */
    int64_t threads, batch_size, epochs, nbatches, neg;
    float lr, margin;
    float *ent, *rel, *normv;   /* device tables of this universe */
    float *ent_acc, *rel_acc, *norm_acc;
    int64_t dim;
} pt_universe_job;
/* prepared set: graphs uploaded, per-universe workspace (LCG states, gradient rows, flags) in HBM */
typedef struct pt_universe_set pt_universe_set;
int pt_universe_set_create(const pt_universe_job *jobs, int64_t n, int32_t model, int32_t p_norm, int32_t norm_flag,
                           int32_t opt, int64_t bern, int64_t filter, pt_universe_set **out);
/* run every universe's `epochs` (continuing from the current LCG states); d_losses: NULL or device
 * [sum of epochs] floats, job-order concatenation of Trainer.run's per-epoch loss sums */
int pt_universe_set_train(pt_universe_set *s, float *d_losses, void *stream);
int pt_universe_set_free(pt_universe_set *s);
/* per-universe cycle counters of the fast kernel (on = 1; off by default) and their readout: out[n][64], per
 * universe (in the set's launch order) shader-clock cycles spent in epoch presampling, phase A, phase B, the
 * step count, batch size, dim and entity count (last train call); out[.][7]: the universe's start on the 100 MHz
 * wall clock (low 32 bits, in the high word) and its duration in those ticks (low word); out[.][63]: where it ran -
 * its XCD (high word) and the workgroup's HW_REG_HW_ID (low word: CU, SH, SE fields); team universes: out[.][60]
 * width << 32 | one-XCD flag, [61] member 0's barrier cycles, [62] member 0's phase-B rows summed over the steps; the
 * other words of out[.][8..59]: phase stamps of one step of lane group 0 in the measurement build (make TUNING=1),
 * zero otherwise */
int pt_universe_set_profiling(pt_universe_set *s, int32_t on);
/* Team universes (csrc/universes_team.h), process-wide and read when a set is created: when a set holds fewer
 * universes than the GPU has CUs, the spare CUs train its longest universes with teams of up to `w` workgroups
 * (one step's positives and row updates split over the members; 1, 2 or 4; default 1: one workgroup each - teams
 * measured slower than one workgroup, round 6) */
int pt_set_universe_team_width(int32_t w);
int32_t pt_get_universe_team_width(void);
/* universes of set s trained by teams, and the workgroups their launches take */
int pt_universe_set_teams(const pt_universe_set *s, int64_t *team_universes, int64_t *team_workgroups);
int pt_universe_set_profile(pt_universe_set *s, uint64_t *out);
/* the current LCG states of job `job` (input order) of a set: `threads` values (host copy; synchronizes) */
int pt_universe_set_states(pt_universe_set *s, int64_t job, uint64_t *out);
/* every job's LCG states back to their values at pt_universe_set_create (re-running the same trainings from the
 * same start, e.g. a benchmark's repeats; the caller restores tables and optimizer state) */
int pt_universe_set_reset(pt_universe_set *s);
/* the concurrent class launches of the last fast-path train call: *n_out = their count; out (when not NULL,
 * cap >= count): per launch {start ms, end ms, universes}, times relative to the earliest start (HIP timing events
 * on each launch's stream). The launches run on process-wide streams with hardware queues of their own, so they
 * overlap regardless of the caller's own streams. */
int pt_universe_set_launch_times(pt_universe_set *s, int64_t cap, float *out, int64_t *n_out);
/* 1 when universes of embedding dim `dim` train on the fast universe kernels (model PT_TRANSE / PT_TRANSH),
 * else 0 (pt_universe_set_create then fails with PT_EINVAL). No device call. */
int pt_universe_dim_supported(int64_t dim, int32_t model);
/* reference-order (deterministic) mode of a set (see pt_trainer_set_deterministic): one workgroup per
 * universe runs its steps with the ordered per-row sums; its workspace is allocated on first use */
int pt_universe_set_deterministic(pt_universe_set *s, int32_t on);
/* create + train + free (synchronizes `stream`) */
int pt_universes_train(const pt_universe_job *jobs, int64_t n, int32_t model, int32_t p_norm, int32_t norm_flag,
                       int32_t opt, int64_t bern, int64_t filter, float *d_losses, void *stream);
enum { PT_DETERMINISTIC = 1 };
/* the same with flags (PT_DETERMINISTIC: reference-order mode) */
int pt_universes_train_ex(const pt_universe_job *jobs, int64_t n, int32_t model, int32_t p_norm, int32_t norm_flag,
                          int32_t opt, int64_t bern, int64_t filter, int32_t flags, float *d_losses, void *stream);

/* Initial tables of universe models drawn on the GPU, bit-identical to the torch CPU generator after
 * torch.manual_seed(seed): the reference builds each universe's TransE / TransH on the CPU after
 * set_random_seed(seed0 + k) (Parallel_Universe_Config.py:157-161, 169-177; nn.Embedding's normal_ draws, then
 * xavier_uniform_, TransE.py:17-36, TransH.py:17-42). A job skips `skip` 32-bit outputs of MT19937(seed mod 2^32) -
 * the draws the constructor's normal_ calls consume (the caller counts them) - then fills its `ntab` tables in
 * order, one output per element: out = (float)((x & 0xffffff) * 2^-24 * ((float)hi - (float)lo) + (float)lo) in
 * double (torch's float uniform_). Tables are device buffers of numel floats; the call synchronizes `stream`. */
typedef struct {
    uint64_t seed;
    int64_t skip;
    int32_t ntab;
    int32_t pad_;
    int64_t numel[4];
    double lo[4], hi[4];
    float *out[4];
} pt_torch_init_job;
int pt_torch_init_tables(const pt_torch_init_job *jobs, int64_t n, void *stream);

/* ------------------------------------------------------------------ link prediction --------- */
/* Per-universe all-entity scoring with a float MIN reduction into per-key rows
 * (obtain_embedding_space_score + transmit_max_scores, Parallel_Universe_Config.py:446-465, :516-543).
 * d_key_rows: [n_keys][global_ent_total] fp32 device buffer (init +inf). A pair names one universe
 * holding both the key's anchor entity and relation: every local entity e of that universe is scored
 * as the missing side (side 0: head prediction, (e, r, anchor); side 1: tail prediction, (anchor, r, e);
 * the same side convention as pt_rank_queries / pt_known_partners)
 * and MIN-reduced into row `key` at column ent_remap[e]. Universes of different dims may be mixed. */
typedef struct {
    const float *ent, *rel, *normv;        /* device tables of the universe */
    int64_t ent_total, rel_total, dim;
    const int64_t *d_ent_remap;            /* device, length ent_total (local -> global) */
} pt_lp_universe;
typedef struct {
    int32_t key, universe, anchor, rel, side;   /* anchor / rel are universe-LOCAL ids */
} pt_lp_pair;
/* The pairs above for every key and universe (host only; the universes eval_universes scores per key,
 * Parallel_Universe_Config.py:470-476): universe u (< 2^31) holds the global entities ent_ids[ent_off[u] ..
 * ent_off[u + 1]) and relations rel_ids[rel_off[u] .. rel_off[u + 1]) in local order; key k is (key_side[k],
 * key_anchor[k], key_rel[k]) in global ids. Rows (k, u, local anchor, local relation, side) for every u holding
 * both, ordered by key then universe. With out == NULL *n_out is an upper bound on the rows (the keys' anchor
 * occurrences); with out, *n_out is the rows written (PT_EINVAL if more than cap). */
int pt_lp_pairs(int64_t n, const int64_t *ent_off, const int64_t *ent_ids, const int64_t *rel_off,
                const int64_t *rel_ids, int64_t n_keys, const int64_t *key_anchor, const int64_t *key_rel,
                const int64_t *key_side, pt_lp_pair *out, int64_t cap, int64_t *n_out);
int pt_lp_min_scores(const pt_lp_universe *us, int64_t n_universes, int32_t model, int32_t p_norm,
                     int32_t norm_flag, const pt_lp_pair *pairs, int64_t n_pairs, int64_t global_ent_total,
                     float *d_key_rows, float *d_key_tuple, void *stream);
/* d_key_tuple (optional, [n_keys], init +inf): MIN over the pairs' universes of the null_vector score
 * _calc(anchor, 0, r) / _calc(0, anchor, r) on the raw anchor row (calc_tuple_score,
 * Parallel_Universe_Config.py:405-416, transmit_tuple_max_score :494-514) */

/* Ranks straight from global-order score rows (device): query q is ranked on row d_row_of[q] with
 * truth entity d_truth[q]; +inf entries are replaced by d_repl[q] when d_repl is non-NULL
 * (missing_embedding_handling = 'null_vector'); d_part_off/d_part = CSR of the known partners of the
 * query's (anchor, r) (pt_known_partners). Same raw / filtered counts as testHead/testTail on the
 * candidate-order vector (Test.h:118-359) and validHead/validTail (Valid.h:117-240). */
int pt_rank_rows(const float *d_rows, int64_t ent_total, const int64_t *d_row_of, const int64_t *d_truth,
                 const float *d_repl, const int64_t *d_part_off, const int64_t *d_part, int64_t n, int64_t *d_raw,
                 int64_t *d_filt, void *stream);
/* Type-constrained raw / filtered counts of the same queries (testHead/testTail with type_constrain,
 * Test.h:127-130, :168-178, :288-298; replaces that branch of the symbols bound at Tester.py:80-82):
 * d_rel[q] selects the relation's type list [d_type_lef[r], d_type_rig[r]) of d_types (ascending, as
 * importTypeFiles sorts it, Reader.h:352-396); d_part must be ascending per query (pt_known_partners
 * returns it so). The reference's position/entity quirk is kept: type entity j is compared with the
 * score at candidate position j. */
int pt_rank_types(const float *d_rows, int64_t ent_total, const int64_t *d_row_of, const int64_t *d_truth,
                  const float *d_repl, const int64_t *d_rel, const int64_t *d_type_lef, const int64_t *d_type_rig,
                  const int64_t *d_types, const int64_t *d_part_off, const int64_t *d_part, int64_t n,
                  int64_t *d_raw, int64_t *d_filt, void *stream);

/* Filtered / raw ranks (testHead/testTail, Test.h:118-359) for many queries at once on host threads:
 * con rows [n][ent_total] in candidate order, anchors per query. Known-triple set from
 * pt_known_create (tripleList, Reader.h:246-342). */
typedef struct pt_known pt_known;
int pt_known_create(const int64_t *h, const int64_t *t, const int64_t *r, int64_t n, pt_known **out);
int pt_known_free(pt_known *k);
/* CSR of the known partners of (anchor[q], rel[q]): side 0 = heads h of known (h, anchor, r), side 1 =
 * tails t of known (anchor, t, r). off has n + 1 entries; with list == NULL only the offsets are filled. */
int pt_known_partners(const pt_known *k, int32_t side, int64_t n, const int64_t *anchor, const int64_t *rel,
                      int64_t *off, int64_t *list);
int pt_rank_queries(const pt_known *k, int64_t ent_total, const int64_t *h, const int64_t *t, const int64_t *r,
                    int64_t n, int32_t side, const float *con, int64_t *raw, int64_t *filt, int64_t n_workers);

/* Checkpoint encoding of the universe id maps (host only; save_parameters, Parallel_Universe_Config.py:890-899,
 * writes the reference's dictionaries filled by process_universe_mappings, :179-207). Universes uids[u]
 * (ascending, < 2^31) hold the global ids ids[off[u] .. off[u + 1]) in local order (< 2^31). Each call writes the
 * item region of a protocol-4 pickle stream (the part between MARK and SETITEMS that
 * openke/config/_map_pickle.py wraps with the container header); with out == NULL only *n_out (bytes) is set.
 * pt_pickle_id_maps: per universe the pair uid: defaultdict(int){ids[off[u] + i]: i} (memo 0 / 1 must hold
 * collections.defaultdict / builtins.int). pt_pickle_universe_sets: per global id, in order of first
 * appearance, the pair id: {universes holding it} (EMPTY_SET + ADDITEMS, universe order). */
int pt_pickle_id_maps(int64_t n, const int64_t *uids, const int64_t *off, const int64_t *ids, uint8_t *out,
                      int64_t cap, int64_t *n_out);
int pt_pickle_universe_sets(int64_t n, const int64_t *uids, const int64_t *off, const int64_t *ids, uint8_t *out,
                            int64_t cap, int64_t *n_out);

/* Checkpoint archive (host only; the file torch.save writes, read back by torch.load - save_parameters,
 * Parallel_Universe_Config.py:890-899): records[i] (name with the archive folder, e.g. "ckpt/data.pkl", data,
 * size) stored in order, each record's data on an `alignment` boundary (a power of two; torch uses 64), ZIP64 where
 * a size, offset or the count needs it (force_zip64: everywhere). CRC-32s of records with crc_known == 0 are
 * computed on up to `threads` threads and written back (crc_known = 1), so an immutable record's CRC can be
 * reused by a later archive. Runs without the Python GIL when called through ctypes. PT_EIO on a file error. */
typedef struct {
    const char *name;
    const void *data;
    int64_t size;
    uint32_t crc32;
    int32_t crc_known;
} pt_zip_record;
int pt_zip_write(const char *path, pt_zip_record *records, int64_t n, int32_t alignment, int32_t threads,
                 int32_t force_zip64);

/* The sampler of the Base.so-compatible global context below (its LCG states follow setRandomSeed /
 * randReset and its graph follows importTrainFiles / swapHelpers), so pt_trainer_* can train on exactly
 * the batch stream the reference's TrainDataLoader.sampling() would produce. */
pt_sampler *pt_legacy_sampler(void);
/* PT_OK or the error of the last importTrainFiles / importTestFiles (which return void like the
 * reference's and leave the previous data in place on failure; pt_last_error() has the message). */
int pt_legacy_import_status(void);
int64_t pt_legacy_bern(void);
/* test (valid = 0) or valid (valid = 1) triples of the global context in ranking order; returns the
 * count, fills the arrays when non-NULL. The known-triple set used by the filtered rank. */
int64_t pt_legacy_eval_triples(int32_t valid, int64_t *h, int64_t *t, int64_t *r);
const pt_known *pt_legacy_known(void);
/* the type lists importTypeFiles loaded (side 0 heads, 1 tails): lef/rig per relation (relTotal entries)
 * and the lists, ascending per relation; returns the list length, -1 before importTypeFiles */
int64_t pt_legacy_types(int32_t side, int64_t *lef, int64_t *rig, int64_t *list);
/* the global context's full training graph (importTrainFiles), e.g. for pt_universe_build_many */
pt_graph *pt_legacy_graph(void);

/* ------------------------------------------------------------------ B: Base.so-compatible ---- */
/* Same names and semantics as the reference (see file:line per symbol in DESIGN.md §Boundary). */
void setInPath(char *path);                          /* Setting.h:12-19 */
void setOutPath(char *path);                         /* Setting.h:21-28 */
void setWorkThreads(int64_t threads);                /* Setting.h:36-39 */
int64_t getWorkThreads(void);                        /* Setting.h:41-44 */
void setBern(int64_t con);                           /* Setting.h:92-95 */
void setRandomSeed(int64_t seed);                    /* Random.h:37-42 */
int64_t getRandomSeed(void);                         /* Random.h:44-47 */
void randReset(void);                                /* Random.h:10-15 */
void importTrainFiles(void);                         /* Reader.h:169-234 */
int64_t getEntityTotal(void);                        /* Setting.h:57-60 */
int64_t getRelationTotal(void);                      /* Setting.h:62-65 */
int64_t getTrainTotal(void);                         /* Setting.h:72-75 */
int64_t getTestTotal(void);                          /* Setting.h:77-80 */
int64_t getValidTotal(void);                         /* Setting.h:82-85 */
int64_t getTripleTotal(void);                        /* Setting.h:67-70 */
/* Base.cpp:266-279 — host buffers; batch built on the GPU, copied back */
void sampling(int64_t *batch_h, int64_t *batch_t, int64_t *batch_r, float *batch_y, int64_t batchSize,
              int64_t negRate, int64_t negRelRate, int64_t mode, int64_t filter_flag, int64_t p, int64_t val_loss);
void getParallelUniverse(int64_t triple_constraint, float balance_parameter);   /* UniverseConstructor.h:327 */
int64_t getEntityTotalUniverse(void);                /* UniverseSetting.h:64-67 */
int64_t getRelationTotalUniverse(void);              /* UniverseSetting.h:69-72 */
int64_t getTrainTotalUniverse(void);                 /* UniverseSetting.h:74-77 */
void getEntityRemapping(int64_t *ent_remapping);     /* UniverseSetting.h:79-84 */
void getRelationRemapping(int64_t *rel_remapping);   /* UniverseSetting.h:86-91 */
void swapHelpers(void);                              /* UniverseSetting.h:123-154 */
/* neighbourhood getters (Base.cpp:312-466; bound at TrainDataLoader.py:60-101, used by
 * get_positive_entities / get_negative_entities / get_entity_relations, :248-276) */
int64_t getNumOfNegatives(int64_t entity, int64_t relation, int64_t entity_is_tail);
int64_t getNumOfPositives(int64_t entity, int64_t relation, int64_t entity_is_tail);
void getNegativeEntities(int64_t *out, int64_t entity, int64_t relation, int64_t entity_is_tail);
void getPositiveEntities(int64_t *out, int64_t entity, int64_t relation, int64_t entity_is_tail);
int64_t getNumOfEntityRelations(int64_t entity, int64_t entity_is_tail);
void getEntityRelations(int64_t *out, int64_t entity, int64_t entity_is_tail);
void resetUniverse(void);                            /* UniverseSetting.h:160-190 */
void activateLoadOfAllTriples(int64_t flag);         /* Reader.h:241-244 */
void importTestFiles(void);                          /* Reader.h:246-342 */
void importTypeFiles(void);                          /* Reader.h:344-396 */
void initTest(void);                                 /* Test.h:23-35 */
void getHeadBatch(int64_t *ph, int64_t *pt, int64_t *pr);    /* Test.h:37-71 */
void getTailBatch(int64_t *ph, int64_t *pt, int64_t *pr);    /* Test.h:73-107 */
/* triple classification (TestDataLoader.sampling_tc): the test triples and one negative each, the coin
 * and the filtered corruption drawn from sampler thread 0 (getNegTest + getTestBatch, Test.h:576-599) */
void getTestBatch(int64_t *ph, int64_t *pt, int64_t *pr, int64_t *nh, int64_t *nt, int64_t *nr);
void testHead(float *con, int64_t lastHead, int64_t type_constrain);   /* Test.h:118-238 */
void testTail(float *con, int64_t lastTail, int64_t type_constrain);   /* Test.h:240-359 */
void test_link_prediction(int64_t type_constrain);   /* Test.h:398-504 */
float getTestLinkMRR(int64_t type_constrain);        /* Test.h:562-567 */
float getTestLinkMR(int64_t type_constrain);         /* Test.h:555-560 */
float getTestLinkHit10(int64_t type_constrain);      /* Test.h:533-539 */
float getTestLinkHit3(int64_t type_constrain);       /* Test.h:541-546 */
float getTestLinkHit1(int64_t type_constrain);       /* Test.h:548-553 */
void validInit(void);                                /* Valid.h */
void getValidHeadBatch(int64_t *ph, int64_t *pt, int64_t *pr);
void getValidTailBatch(int64_t *ph, int64_t *pt, int64_t *pr);
void validHead(float *con, int64_t lastHead);
void validTail(float *con, int64_t lastTail);
float getValidHit10(void);

#ifdef __cplusplus
}
#endif
#endif
