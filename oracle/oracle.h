/*
 * CPU ORACLE — test infrastructure only.
 *
 * A plain-C restatement of the reference's hot path (luofeisg/OpenKE-PuTransE), used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER. Nothing in the product
 * (openke-putranse_amd/) links, loads or calls it.
 *
 * Parity pinning: every function below is checked in tests/test_oracle.py against golden vectors
 * produced by the reference itself (tests/golden/make_golden.py imports the reference Python and the
 * reference C++ core compiled from its own sources into oracle/_ref/Base.so).
 */
#ifndef PUTRANSE_ORACLE_H
#define PUTRANSE_ORACLE_H
#include <stdint.h>

/* glibc srand()/rand() (TYPE_3 additive feedback generator) restated with private state.
 * The reference seeds its sampler and its universe walk from glibc rand() (Random.h:10-15, :32-45). */
typedef struct {
    int32_t state[31];
    int f, r;
} orand_t;
void orand_seed(orand_t *g, uint32_t seed);
int32_t orand_next(orand_t *g);

/* Training graph with the reference's helper indices (Reader.h:58-234, UniverseConstructor.h:235-325). */
typedef struct { int64_t h, r, t; } otriple;
typedef struct {
    int64_t ent_total, rel_total, train_total;
    otriple *train_list, *train_head, *train_tail, *train_rel, *train_rel2;
    int64_t *lef_head, *rig_head, *lef_tail, *rig_tail, *lef_rel, *rig_rel, *lef_rel2, *rig_rel2;
    int64_t *freq_ent, *freq_rel;
    float *left_mean, *right_mean;
} okg;

okg *okg_load(const char *dir);                      /* importTrainFiles, Reader.h:169-234 */
void okg_free(okg *g);
int64_t okg_ent_total(const okg *g);
int64_t okg_rel_total(const okg *g);
int64_t okg_train_total(const okg *g);
void okg_get_train(const okg *g, int64_t *h, int64_t *t, int64_t *r);
float okg_left_mean(const okg *g, int64_t r);
float okg_right_mean(const okg *g, int64_t r);

/* randReset (Random.h:10-15): next_random[i] = rand() */
void oracle_rand_reset(orand_t *g, int64_t threads, uint64_t *states);
/* sampling + getBatch, mode 0, neg_rel 0 (Base.cpp:185-310) */
void oracle_sampling(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t bern,
                     int64_t filter, int64_t *h, int64_t *t, int64_t *r, float *y);
void oracle_sampling_sides(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t bern,
                           int64_t filter, int64_t *h, int64_t *t, int64_t *r, float *y, int8_t *side);
/* sampling with mode (0 / -1 sampling_head / 1 sampling_tail) and neg_rel relation corruptions
 * (Base.cpp:185-264, Corrupt.h:108-189); seq = bs * (1 + neg + neg_rel) */
void oracle_sampling_ex(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t neg_rel,
                        int64_t mode, int64_t bern, int64_t filter, int64_t *h, int64_t *t, int64_t *r, float *y);

/* getParallelUniverse (UniverseConstructor.h:327-397): returns the universe graph (local ids, helpers
 * built as loadUniverseHelpers does) and writes local->global maps (sized >= E and >= R). */
okg *oracle_universe(const okg *g, orand_t *rng, int64_t tc, float balance, int64_t *ent_remap, int64_t *rel_remap);

/* One minibatch-synchronous training step on a sampled batch: forward (TransE.py:46-74 /
 * TransH.py:52-93), MarginLoss (MarginLoss.py:24-28), autograd-equivalent backward and a dense
 * SGD / Adagrad update (Trainer.py:62-88). Tables are updated in place; returns the loss. */
float oracle_train_step(int model, int p_norm, int norm_flag, int opt, float lr, float margin, int64_t ent_total,
                        int64_t rel_total, int64_t dim, float *ent, float *rel, float *normv, float *ent_acc,
                        float *rel_acc, float *norm_acc, const int64_t *h, const int64_t *t, const int64_t *r,
                        int64_t bs, int64_t neg);

/* The same step on `workers` threads (scores, per-slot gradient rows and per-row sums in parallel; every
 * float sum keeps its order, so the result is bit-identical to oracle_train_step). */
float oracle_train_step_mt(int model, int p_norm, int norm_flag, int opt, float lr, float margin, int64_t ent_total,
                           int64_t rel_total, int64_t dim, float *ent, float *rel, float *normv, float *ent_acc,
                           float *rel_acc, float *norm_acc, const int64_t *h, const int64_t *t, const int64_t *r,
                           int64_t bs, int64_t neg, int64_t workers);

/* Test infrastructure (tests/helpers.py kappa_bound): per table element the step's gradient summed in the
 * reference's order, the sum of its contributions' magnitudes and its absolute-value evaluation; per row the
 * contribution count and a near-tie flag (no update). Outputs [E + R (+ R for TransH)][d] (entity, relation,
 * norm_vector rows) and [E + R (+ R)]; returns the loss. */
float oracle_grad_mass(int model, int p, int norm_flag, float margin, int64_t E, int64_t R, int64_t d, float *ent,
                       float *rel, float *normv, const int64_t *h, const int64_t *t, const int64_t *r, int64_t bs,
                       int64_t neg, float *gsum, float *gmass, float *gabs, int32_t *gcnt, int32_t *gtie);

/* Scores as model.predict(...) computes them; mode 0 normal, 1 head_batch, 2 tail_batch (TransE.py:46-60). */
void oracle_score(int model, int p_norm, int norm_flag, int mode, int64_t dim, const float *ent, const float *rel,
                  const float *normv, const int64_t *h, const int64_t *t, const int64_t *r, int64_t n, float *out);

/* Link prediction ranking (Test.h:118-359, :398-504). triples: test+train+valid (h,t,r) rows, any order;
 * test rows are ranked in cmp_rel2 order as importTestFiles sorts them. con_head/con_tail:
 * [test_total][ent_total] score rows already in candidate order (getHeadBatch/getTailBatch).
 * Outputs raw/filtered ranks per test row (0-based counts, as the reference's l_s / l_filter_s) and
 * metrics[5] = {mrr, mr, hit10, hit3, hit1} (filtered, float accumulation as the reference). */
void oracle_sort_test(int64_t n, int64_t *h, int64_t *t, int64_t *r);
void oracle_link_prediction(int64_t ent_total, const int64_t *all_h, const int64_t *all_t, const int64_t *all_r,
                            int64_t n_all, const int64_t *test_h, const int64_t *test_t, const int64_t *test_r,
                            int64_t n_test, const float *con_head, const float *con_tail, int64_t *rank_head,
                            int64_t *frank_head, int64_t *rank_tail, int64_t *frank_tail, float *metrics);

/* metrics[5] from filtered ranks alone (the accumulation of oracle_link_prediction) */
void oracle_metrics_from_ranks(int64_t n_test, const int64_t *frank_head, const int64_t *frank_tail, float *metrics);

/* Reference-faithful sequential step timing helper for bench.py's cpu_baseline leg: samples and trains
 * `steps` steps with the restated sampler + step (single thread). Returns total slots processed. */
int64_t oracle_train_loop(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t bern,
                          int64_t filter, int model, int p_norm, int norm_flag, int opt, float lr, float margin,
                          int64_t dim, float *ent, float *rel, float *normv, float *ent_acc, float *rel_acc,
                          float *norm_acc, int64_t steps);
/* the same loop with the sampler slices and the step phases on `workers` threads (bit-identical results);
 * losses (optional) receives each step's loss */
int64_t oracle_train_loop_mt(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t bern,
                             int64_t filter, int model, int p_norm, int norm_flag, int opt, float lr, float margin,
                             int64_t dim, float *ent, float *rel, float *normv, float *ent_acc, float *rel_acc,
                             float *norm_acc, int64_t steps, int64_t workers, float *losses);
/* type-constrained counts and metrics of testHead/testTail/test_link_prediction (Test.h:127-502); type
 * lists per relation [lef, rig) as importTypeFiles builds them (Reader.h:352-396) */
void oracle_rank_constrained(int64_t E, const int64_t *ah, const int64_t *at, const int64_t *ar, int64_t n_all,
                             const int64_t *th, const int64_t *tt, const int64_t *tr, int64_t n_test,
                             const float *con_head, const float *con_tail, const int64_t *head_lef,
                             const int64_t *head_rig, const int64_t *head_type, const int64_t *tail_lef,
                             const int64_t *tail_rig, const int64_t *tail_type, int64_t *rank_head,
                             int64_t *frank_head, int64_t *rank_tail, int64_t *frank_tail, float *metrics);

#endif
