/*
 * CPU ORACLE — test infrastructure only (see oracle.h). Restates the reference algorithm; each
 * function cites the reference file:line it follows. Parity is pinned by tests/test_oracle.py
 * against fixtures produced by the reference itself (tests/golden/make_golden.py).
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- glibc rand (TYPE_3) ----------- */
/* glibc stdlib/random_r.c: srandom_r seeds 31 words with 16807*x mod (2^31-1) (Schrage form), sets
 * the feedback pointers 3 apart and discards 310 outputs; random_r adds the two taps and returns
 * the sum >> 1. The reference calls it through srand()/rand() (Random.h:37-45, :32-34). */
void orand_seed(orand_t *g, uint32_t seed) {
    if (seed == 0) seed = 1;
    int32_t word = (int32_t)seed;
    g->state[0] = word;
    for (int i = 1; i < 31; ++i) {
        long hi = word / 127773;
        long lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        g->state[i] = word;
    }
    g->f = 3;
    g->r = 0;
    for (int i = 0; i < 310; ++i) (void)orand_next(g);
}

int32_t orand_next(orand_t *g) {
    uint32_t val = (uint32_t)g->state[g->f] + (uint32_t)g->state[g->r];
    g->state[g->f] = (int32_t)val;
    int32_t result = (int32_t)(val >> 1);
    if (++g->f >= 31) {
        g->f = 0;
        ++g->r;
    } else if (++g->r >= 31) {
        g->r = 0;
    }
    return result;
}

/* rand(a,b) = rand() % (b-a) + a   (Random.h:32-34) */
static int64_t orand_range(orand_t *g, int64_t a, int64_t b) { return (int64_t)orand_next(g) % (b - a) + a; }

/* ---------------------------------------------------------------- per-thread LCG --------------- */
/* randd / rand_max (Random.h:18-29) */
static inline uint64_t lcg_next(uint64_t *s) {
    *s = *s * 25214903917ULL + 11ULL;
    return *s;
}
static inline int64_t lcg_max(uint64_t *s, int64_t x) { return (int64_t)(lcg_next(s) % (uint64_t)x); }

void oracle_rand_reset(orand_t *g, int64_t threads, uint64_t *states) {
    for (int64_t i = 0; i < threads; ++i) states[i] = (uint64_t)(int64_t)orand_next(g);
}

/* ---------------------------------------------------------------- graph + helpers -------------- */
static int cmp_head(const void *a, const void *b) {   /* Triple.h:7-9 */
    const otriple *x = a, *y = b;
    if (x->h != y->h) return x->h < y->h ? -1 : 1;
    if (x->r != y->r) return x->r < y->r ? -1 : 1;
    if (x->t != y->t) return x->t < y->t ? -1 : 1;
    return 0;
}
static int cmp_tail(const void *a, const void *b) {   /* Triple.h:11-13 */
    const otriple *x = a, *y = b;
    if (x->t != y->t) return x->t < y->t ? -1 : 1;
    if (x->r != y->r) return x->r < y->r ? -1 : 1;
    if (x->h != y->h) return x->h < y->h ? -1 : 1;
    return 0;
}
static int cmp_rel(const void *a, const void *b) {    /* Triple.h:15-17 */
    const otriple *x = a, *y = b;
    if (x->h != y->h) return x->h < y->h ? -1 : 1;
    if (x->t != y->t) return x->t < y->t ? -1 : 1;
    if (x->r != y->r) return x->r < y->r ? -1 : 1;
    return 0;
}
static int cmp_rel2(const void *a, const void *b) {   /* Triple.h:19-21 */
    const otriple *x = a, *y = b;
    if (x->r != y->r) return x->r < y->r ? -1 : 1;
    if (x->h != y->h) return x->h < y->h ? -1 : 1;
    if (x->t != y->t) return x->t < y->t ? -1 : 1;
    return 0;
}

static int64_t count_lines(FILE *f) {                 /* Utilities.h:47-57 */
    int64_t n = 0;
    int c;
    while ((c = getc(f)) != EOF)
        if (c == '\n') ++n;
    rewind(f);
    return n;
}

static int64_t *alloc_i64(int64_t n, int fill_minus_one) {
    int64_t *p = calloc((size_t)(n > 0 ? n : 1), sizeof(int64_t));
    if (fill_minus_one) memset(p, -1, sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
    return p;
}

/* Builds the four sorted copies, the [lef,rig] ranges and left/right means. `universe_form` selects
 * loadUniverseHelpers (UniverseConstructor.h:235-325: rig arrays -1 only on [0,E_u), freqRel from the
 * list itself) over loadHelpers (Reader.h:58-167). Both give identical arrays on a deduplicated list. */
static void build_helpers(okg *g) {
    int64_t n = g->train_total, E = g->ent_total, R = g->rel_total;
    qsort(g->train_list, (size_t)n, sizeof(otriple), cmp_head);
    g->train_head = malloc(sizeof(otriple) * (size_t)(n ? n : 1));
    g->train_tail = malloc(sizeof(otriple) * (size_t)(n ? n : 1));
    g->train_rel = malloc(sizeof(otriple) * (size_t)(n ? n : 1));
    g->train_rel2 = malloc(sizeof(otriple) * (size_t)(n ? n : 1));
    g->freq_ent = alloc_i64(E, 0);
    g->freq_rel = alloc_i64(R, 0);
    for (int64_t i = 0; i < n; ++i) {
        g->train_head[i] = g->train_tail[i] = g->train_rel[i] = g->train_rel2[i] = g->train_list[i];
        g->freq_ent[g->train_list[i].h]++;
        g->freq_ent[g->train_list[i].t]++;
        g->freq_rel[g->train_list[i].r]++;
    }
    qsort(g->train_head, (size_t)n, sizeof(otriple), cmp_head);
    qsort(g->train_tail, (size_t)n, sizeof(otriple), cmp_tail);
    qsort(g->train_rel, (size_t)n, sizeof(otriple), cmp_rel);
    qsort(g->train_rel2, (size_t)n, sizeof(otriple), cmp_rel2);
    g->lef_head = alloc_i64(E, 0); g->rig_head = alloc_i64(E, 1);
    g->lef_tail = alloc_i64(E, 0); g->rig_tail = alloc_i64(E, 1);
    g->lef_rel = alloc_i64(E, 0);  g->rig_rel = alloc_i64(E, 1);
    g->lef_rel2 = alloc_i64(R, 0); g->rig_rel2 = alloc_i64(R, 1);
    for (int64_t i = 1; i < n; ++i) {
        if (g->train_tail[i].t != g->train_tail[i - 1].t) {
            g->rig_tail[g->train_tail[i - 1].t] = i - 1;
            g->lef_tail[g->train_tail[i].t] = i;
        }
        if (g->train_head[i].h != g->train_head[i - 1].h) {
            g->rig_head[g->train_head[i - 1].h] = i - 1;
            g->lef_head[g->train_head[i].h] = i;
        }
        if (g->train_rel[i].h != g->train_rel[i - 1].h) {
            g->rig_rel[g->train_rel[i - 1].h] = i - 1;
            g->lef_rel[g->train_rel[i].h] = i;
        }
        if (g->train_rel2[i].r != g->train_rel2[i - 1].r) {
            g->rig_rel2[g->train_rel2[i - 1].r] = i - 1;
            g->lef_rel2[g->train_rel2[i].r] = i;
        }
    }
    if (n > 0) {
        g->lef_head[g->train_head[0].h] = 0;
        g->rig_head[g->train_head[n - 1].h] = n - 1;
        g->lef_tail[g->train_tail[0].t] = 0;
        g->rig_tail[g->train_tail[n - 1].t] = n - 1;
        g->lef_rel[g->train_rel[0].h] = 0;
        g->rig_rel[g->train_rel[n - 1].h] = n - 1;
        g->lef_rel2[g->train_rel2[0].r] = 0;
        g->rig_rel2[g->train_rel2[n - 1].r] = n - 1;
    }
    g->left_mean = calloc((size_t)(R ? R : 1), sizeof(float));
    g->right_mean = calloc((size_t)(R ? R : 1), sizeof(float));
    for (int64_t i = 0; i < E; ++i) {
        for (int64_t j = g->lef_head[i] + 1; j <= g->rig_head[i]; ++j)
            if (g->train_head[j].r != g->train_head[j - 1].r) g->left_mean[g->train_head[j].r] += 1.0f;
        if (g->lef_head[i] <= g->rig_head[i]) g->left_mean[g->train_head[g->lef_head[i]].r] += 1.0f;
        for (int64_t j = g->lef_tail[i] + 1; j <= g->rig_tail[i]; ++j)
            if (g->train_tail[j].r != g->train_tail[j - 1].r) g->right_mean[g->train_tail[j].r] += 1.0f;
        if (g->lef_tail[i] <= g->rig_tail[i]) g->right_mean[g->train_tail[g->lef_tail[i]].r] += 1.0f;
    }
    for (int64_t i = 0; i < R; ++i) {
        g->left_mean[i] = (float)g->freq_rel[i] / g->left_mean[i];
        g->right_mean[i] = (float)g->freq_rel[i] / g->right_mean[i];
    }
}

okg *okg_load(const char *dir) {                      /* importTrainFiles, Reader.h:169-234 */
    char path[4096];
    okg *g = calloc(1, sizeof(okg));
    snprintf(path, sizeof path, "%srelation2id.txt", dir);
    FILE *f = fopen(path, "r");
    if (!f) { free(g); return NULL; }
    g->rel_total = count_lines(f);
    fclose(f);
    snprintf(path, sizeof path, "%sentity2id.txt", dir);
    f = fopen(path, "r");
    if (!f) { free(g); return NULL; }
    g->ent_total = count_lines(f);
    fclose(f);
    snprintf(path, sizeof path, "%strain2id.txt", dir);
    f = fopen(path, "r");
    if (!f) { free(g); return NULL; }
    int64_t n = count_lines(f);
    g->train_list = calloc((size_t)(n ? n : 1), sizeof(otriple));
    for (int64_t i = 0; i < n; ++i) {
        long a = 0, b = 0, c = 0;
        if (fscanf(f, "%ld %ld %ld", &a, &b, &c) != 3) break;
        g->train_list[i].h = a; g->train_list[i].t = b; g->train_list[i].r = c;
    }
    fclose(f);
    qsort(g->train_list, (size_t)n, sizeof(otriple), cmp_head);
    int64_t m = n ? 1 : 0;
    for (int64_t i = 1; i < n; ++i)
        if (cmp_head(&g->train_list[i], &g->train_list[i - 1]) != 0) g->train_list[m++] = g->train_list[i];
    g->train_total = m;
    build_helpers(g);
    return g;
}

void okg_free(okg *g) {
    if (!g) return;
    free(g->train_list); free(g->train_head); free(g->train_tail); free(g->train_rel); free(g->train_rel2);
    free(g->lef_head); free(g->rig_head); free(g->lef_tail); free(g->rig_tail);
    free(g->lef_rel); free(g->rig_rel); free(g->lef_rel2); free(g->rig_rel2);
    free(g->freq_ent); free(g->freq_rel); free(g->left_mean); free(g->right_mean);
    free(g);
}
int64_t okg_ent_total(const okg *g) { return g->ent_total; }
int64_t okg_rel_total(const okg *g) { return g->rel_total; }
int64_t okg_train_total(const okg *g) { return g->train_total; }
float okg_left_mean(const okg *g, int64_t r) { return g->left_mean[r]; }
float okg_right_mean(const okg *g, int64_t r) { return g->right_mean[r]; }
void okg_get_train(const okg *g, int64_t *h, int64_t *t, int64_t *r) {
    for (int64_t i = 0; i < g->train_total; ++i) {
        h[i] = g->train_list[i].h; t[i] = g->train_list[i].t; r[i] = g->train_list[i].r;
    }
}

/* ---------------------------------------------------------------- negative corruption --------- */
/* corrupt_head / corrupt_tail with filter (Corrupt.h:27-56, :75-104). `heads` selects the head-sorted
 * list (corrupt_head: returns a replacement TAIL avoiding known (h,r,.) tails). */
static int64_t corrupt_filtered(const okg *g, int heads, int64_t key, int64_t r, uint64_t *s) {
    const otriple *L = heads ? g->train_head : g->train_tail;
    const int64_t *lef = heads ? g->lef_head : g->lef_tail, *rig = heads ? g->rig_head : g->rig_tail;
#define VAL(k) (heads ? L[(k)].t : L[(k)].h)
    int64_t lo = lef[key] - 1, hi = rig[key], mid;
    while (lo + 1 < hi) {
        mid = (lo + hi) >> 1;
        if (L[mid].r >= r) hi = mid; else lo = mid;
    }
    int64_t ll = hi;
    lo = lef[key];
    hi = rig[key] + 1;
    while (lo + 1 < hi) {
        mid = (lo + hi) >> 1;
        if (L[mid].r <= r) lo = mid; else hi = mid;
    }
    int64_t rr = lo;
    int64_t tmp = lcg_max(s, g->ent_total - (rr - ll + 1));
    if (tmp < VAL(ll)) return tmp;
    if (tmp > VAL(rr) - rr + ll - 1) return tmp + rr - ll + 1;
    lo = ll;
    hi = rr + 1;
    while (lo + 1 < hi) {
        mid = (lo + hi) >> 1;
        if (VAL(mid) - mid + ll - 1 < tmp) lo = mid; else hi = mid;
    }
    return tmp + lo - ll + 1;
#undef VAL
}

/* unfiltered: uniform over [0,E-1) skipping the PASSED entity (Corrupt.h:18-25, :68-74) */
static int64_t corrupt_plain(const okg *g, int64_t skip, uint64_t *s) {
    int64_t tmp = lcg_max(s, g->ent_total - 1);
    return tmp < skip ? tmp : tmp + 1;
}

/* getBatch (Base.cpp:185-264) for every sampler thread in turn; threads write disjoint slices.
 * side (optional, NULL = not recorded): side[b + (k+1)*bs] = 1 when the coin of Base.cpp:219-222 chose
 * corrupt_head (the TAIL replaced), 0 when it chose corrupt_tail (the head replaced). */
void oracle_sampling_sides(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t bern,
                           int64_t filter, int64_t *h, int64_t *t, int64_t *r, float *y, int8_t *side) {
    for (int64_t id = 0; id < threads; ++id) {
        int64_t lef, rig;
        if (bs % threads == 0) {
            lef = id * (bs / threads);
            rig = (id + 1) * (bs / threads);
        } else {
            lef = id * (bs / threads + 1);
            rig = (id + 1) * (bs / threads + 1);
            if (rig > bs) rig = bs;
        }
        uint64_t *s = &states[id];
        float prob = 500;
        for (int64_t b = lef; b < rig; ++b) {
            int64_t i = lcg_max(s, g->train_total);
            otriple p = g->train_list[i];
            h[b] = p.h; t[b] = p.t; r[b] = p.r; y[b] = 1;
            int64_t last = bs;
            for (int64_t k = 0; k < neg; ++k) {
                if (bern) prob = 1000 * g->right_mean[p.r] / (g->right_mean[p.r] + g->left_mean[p.r]);
                const int tail_side = (float)(lcg_next(s) % 1000) < prob;
                if (side) side[b + last] = (int8_t)tail_side;
                if (tail_side) {
                    h[b + last] = p.h;
                    t[b + last] = filter ? corrupt_filtered(g, 1, p.h, p.r, s) : corrupt_plain(g, p.h, s);
                    r[b + last] = p.r;
                } else {
                    h[b + last] = filter ? corrupt_filtered(g, 0, p.t, p.r, s) : corrupt_plain(g, p.t, s);
                    t[b + last] = p.t;
                    r[b + last] = p.r;
                }
                y[b + last] = -1;
                last += bs;
            }
        }
    }
}

void oracle_sampling(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t bern,
                     int64_t filter, int64_t *h, int64_t *t, int64_t *r, float *y) {
    oracle_sampling_sides(g, states, threads, bs, neg, bern, filter, h, t, r, y, NULL);
}

/* corrupt_rel, p == false, filter_flag == true (Corrupt.h:108-135, :179-189): the (h,t) run [ll,rr] of the
 * cmp_rel-sorted list holds the relations already known between h and t; draw among the others.
 * Returns -1 where the reference divides by zero (every relation is known for (h,t)). */
static int64_t corrupt_rel_filtered(const okg *g, int64_t h, int64_t t, uint64_t *s) {
    const otriple *L = g->train_rel;
    int64_t lo = g->lef_rel[h] - 1, hi = g->rig_rel[h], mid;
    while (lo + 1 < hi) {
        mid = (lo + hi) >> 1;
        if (L[mid].t >= t) hi = mid; else lo = mid;
    }
    const int64_t ll = hi;
    lo = g->lef_rel[h];
    hi = g->rig_rel[h] + 1;
    while (lo + 1 < hi) {
        mid = (lo + hi) >> 1;
        if (L[mid].t <= t) lo = mid; else hi = mid;
    }
    const int64_t rr = lo;
    if (g->rel_total - (rr - ll + 1) <= 0) return -1;
    const int64_t tmp = lcg_max(s, g->rel_total - (rr - ll + 1));
    if (tmp < L[ll].r) return tmp;
    if (tmp > L[rr].r - rr + ll - 1) return tmp + rr - ll + 1;
    lo = ll;
    hi = rr + 1;
    while (lo + 1 < hi) {
        mid = (lo + hi) >> 1;
        if (L[mid].r - mid + ll - 1 < tmp) lo = mid; else hi = mid;
    }
    return tmp + lo - ll + 1;
}

/* getBatch with every argument of sampling() (Base.cpp:185-264), val_loss aside: mode 0 is the coin form
 * above; mode -1 (sampling_head) replaces the head by corrupt_tail, mode 1 (sampling_tail) the tail by
 * corrupt_head - both with corrupt_*'s default filter_flag = true (Base.cpp:233-245, Corrupt.h:9, :59) and
 * no coin draw; then neg_rel relation corruptions per positive (Base.cpp:247-253, p = false). */
void oracle_sampling_ex(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t neg_rel,
                        int64_t mode, int64_t bern, int64_t filter, int64_t *h, int64_t *t, int64_t *r, float *y) {
    for (int64_t id = 0; id < threads; ++id) {
        int64_t lef, rig;
        if (bs % threads == 0) {
            lef = id * (bs / threads);
            rig = (id + 1) * (bs / threads);
        } else {
            lef = id * (bs / threads + 1);
            rig = (id + 1) * (bs / threads + 1);
            if (rig > bs) rig = bs;
        }
        uint64_t *s = &states[id];
        float prob = 500;
        for (int64_t b = lef; b < rig; ++b) {
            int64_t i = lcg_max(s, g->train_total);
            otriple p = g->train_list[i];
            h[b] = p.h; t[b] = p.t; r[b] = p.r; y[b] = 1;
            int64_t last = bs;
            for (int64_t k = 0; k < neg; ++k) {
                h[b + last] = p.h; t[b + last] = p.t; r[b + last] = p.r;
                if (mode == 0) {
                    if (bern) prob = 1000 * g->right_mean[p.r] / (g->right_mean[p.r] + g->left_mean[p.r]);
                    if ((float)(lcg_next(s) % 1000) < prob)
                        t[b + last] = filter ? corrupt_filtered(g, 1, p.h, p.r, s) : corrupt_plain(g, p.h, s);
                    else
                        h[b + last] = filter ? corrupt_filtered(g, 0, p.t, p.r, s) : corrupt_plain(g, p.t, s);
                } else if (mode == -1) {
                    h[b + last] = corrupt_filtered(g, 0, p.t, p.r, s);
                } else {
                    t[b + last] = corrupt_filtered(g, 1, p.h, p.r, s);
                }
                y[b + last] = -1;
                last += bs;
            }
            for (int64_t k = 0; k < neg_rel; ++k) {
                h[b + last] = p.h; t[b + last] = p.t;
                r[b + last] = corrupt_rel_filtered(g, p.h, p.t, s);
                y[b + last] = -1;
                last += bs;
            }
        }
    }
}

/* ---------------------------------------------------------------- universe construction ------- */
typedef struct { int64_t *a; int64_t n, cap; } iset;   /* sorted set, std::set<INT> iteration order */
static void iset_init(iset *s) { s->n = 0; s->cap = 16; s->a = malloc(sizeof(int64_t) * 16); }
static int64_t iset_lb(const iset *s, int64_t v) {
    int64_t lo = 0, hi = s->n;
    while (lo < hi) {
        int64_t m = (lo + hi) / 2;
        if (s->a[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}
static void iset_insert(iset *s, int64_t v) {
    int64_t i = iset_lb(s, v);
    if (i < s->n && s->a[i] == v) return;
    if (s->n == s->cap) { s->cap *= 2; s->a = realloc(s->a, sizeof(int64_t) * (size_t)s->cap); }
    memmove(s->a + i + 1, s->a + i, sizeof(int64_t) * (size_t)(s->n - i));
    s->a[i] = v;
    s->n++;
}
static void iset_erase_at(iset *s, int64_t i) {
    memmove(s->a + i, s->a + i + 1, sizeof(int64_t) * (size_t)(s->n - i - 1));
    s->n--;
}

okg *oracle_universe(const okg *g, orand_t *rng, int64_t tc, float balance, int64_t *ent_remap, int64_t *rel_remap) {
    int64_t ntu = tc;
    otriple *U = calloc((size_t)(tc ? tc : 1), sizeof(otriple));
    int64_t focus = orand_range(rng, 0, g->rel_total);                    /* :336-342 */
    int64_t threshold = (int64_t)(balance * (float)tc);                   /* :343-344 */
    iset S;
    iset_init(&S);
    for (int64_t k = g->lef_rel2[focus]; k < g->rig_rel2[focus] + 1; ++k) {   /* :69-80 */
        iset_insert(&S, g->train_rel2[k].h);
        iset_insert(&S, g->train_rel2[k].t);
    }
    if ((uint64_t)S.n > (uint64_t)threshold) {                            /* get_entity_subset :55-67 */
        iset sub;
        iset_init(&sub);
        while (sub.n < threshold) {
            int64_t idx = (int64_t)((uint64_t)(int64_t)orand_next(rng) % (uint64_t)S.n);
            iset_insert(&sub, S.a[idx]);
            iset_erase_at(&S, idx);
        }
        free(S.a);
        S = sub;
    }
    /* BidirectionalRandomWalk (:92-191) */
    int64_t ui = 0, last_dup = -1, tol = 5, not_inc = 20, last_size = 0;
    iset nsp, uent, urel;
    iset_init(&nsp); iset_init(&uent); iset_init(&urel);
    while (ui < ntu) {
        int64_t i = 0;
        while (i < S.n && ui < ntu) {
            int64_t cur = S.a[i];
            int64_t nh = 0, nr = 0, nt = 0, start = -1;
            int from_head;
            if (orand_next(rng) % 1000 < 500)
                from_head = g->rig_head[cur] != -1 ? 1 : (g->rig_tail[cur] != -1 ? 0 : -1);
            else
                from_head = g->rig_tail[cur] != -1 ? 0 : (g->rig_head[cur] != -1 ? 1 : -1);
            if (from_head == 1) {
                int64_t k = orand_range(rng, g->lef_head[cur], g->rig_head[cur] + 1);
                nh = g->train_head[k].h; nr = g->train_head[k].r; nt = g->train_head[k].t; start = nt;
            } else if (from_head == 0) {
                int64_t k = orand_range(rng, g->lef_tail[cur], g->rig_tail[cur] + 1);
                nh = g->train_tail[k].h; nr = g->train_tail[k].r; nt = g->train_tail[k].t; start = nh;
            }
            int dup = 0;
            for (int64_t q = 0; q < ui; ++q)
                if (U[q].h == nh && U[q].r == nr && U[q].t == nt) { dup = 1; break; }
            if (dup) {
                if (last_dup == cur) tol--; else last_dup = cur;
                if (tol == 0) { tol = 5; i++; }
                continue;
            }
            U[ui].h = nh; U[ui].r = nr; U[ui].t = nt;
            iset_insert(&nsp, start);
            iset_insert(&uent, nt);
            iset_insert(&uent, nh);
            iset_insert(&urel, nr);
            iset_erase_at(&S, i);
            ui++;
        }
        iset tmp = S; S = nsp; nsp = tmp;                                  /* swap, leftovers kept */
        if (ui == last_size) not_inc--; else { last_size = ui; not_inc = 20; }
        if (not_inc == 0) { ntu = ui; break; }
    }
    okg *u = calloc(1, sizeof(okg));
    u->ent_total = uent.n;
    u->rel_total = urel.n;
    u->train_total = ntu;
    free(S.a); free(nsp.a); free(uent.a); free(urel.a);
    /* enumerateTrainUniverseTriples (:193-233): ids by first appearance h, t, r */
    int64_t *emap = alloc_i64(g->ent_total, 1), *rmap = alloc_i64(g->rel_total, 1);
    for (int64_t i = 0; i < g->ent_total; ++i) ent_remap[i] = -1;
    for (int64_t i = 0; i < g->rel_total; ++i) rel_remap[i] = -1;
    int64_t ne = 0, nr = 0;
    u->train_list = calloc((size_t)(ntu ? ntu : 1), sizeof(otriple));
    for (int64_t i = 0; i < ntu; ++i) {
        if (emap[U[i].h] == -1) { emap[U[i].h] = ne; ent_remap[ne++] = U[i].h; }
        u->train_list[i].h = emap[U[i].h];
        if (emap[U[i].t] == -1) { emap[U[i].t] = ne; ent_remap[ne++] = U[i].t; }
        u->train_list[i].t = emap[U[i].t];
        if (rmap[U[i].r] == -1) { rmap[U[i].r] = nr; rel_remap[nr++] = U[i].r; }
        u->train_list[i].r = rmap[U[i].r];
    }
    free(emap); free(rmap); free(U);
    build_helpers(u);                                                      /* loadUniverseHelpers */
    return u;
}

/* ---------------------------------------------------------------- model math ------------------ */
static float vnorm2(const float *x, int64_t d) {
    float s = 0;
    for (int64_t i = 0; i < d; ++i) s += x[i] * x[i];
    return sqrtf(s);
}
static float vdot(const float *a, const float *b, int64_t d) {
    float s = 0;
    for (int64_t i = 0; i < d; ++i) s += a[i] * b[i];
    return s;
}
/* F.normalize(x, 2, -1) = x / max(||x||, 1e-12) */
static float normalize_into(const float *x, float *out, int64_t d) {
    float n = vnorm2(x, d);
    float den = n > 1e-12f ? n : 1e-12f;
    for (int64_t i = 0; i < d; ++i) out[i] = x[i] / den;
    return n;
}
/* backward of F.normalize: (g - xhat (xhat . g)) / n  (zero extra term when n <= eps, clamp_min) */
static void normalize_backward(const float *x, float n, const float *g, float *out, int64_t d) {
    if (n > 1e-12f) {
        float c = vdot(g, x, d) / (n * n);
        for (int64_t i = 0; i < d; ++i) out[i] = (g[i] - x[i] * c) / n;
    } else {
        for (int64_t i = 0; i < d; ++i) out[i] = g[i] / 1e-12f;
    }
}

typedef struct {
    int64_t d;
    float *h, *t, *r, *w;          /* raw rows */
    float *hp, *tp;                /* TransH projected rows */
    float *nh, *nt, *nr, *nw;      /* normalized rows */
    float *v;
    float hn, tn, rn, wn, hpn, tpn, hdot, tdot;
} slot_ws;

/* forward of one triple; returns the score, leaves intermediates in ws (TransE.py:46-60, TransH.py:68-93) */
static float slot_forward(int model, int p, int norm_flag, int mode, slot_ws *ws, const float *he, const float *te,
                          const float *re, const float *we) {
    int64_t d = ws->d;
    const float *h = he, *t = te;
    if (model == 1) {
        ws->wn = normalize_into(we, ws->nw, d);
        ws->hdot = vdot(he, ws->nw, d);
        ws->tdot = vdot(te, ws->nw, d);
        for (int64_t i = 0; i < d; ++i) {
            ws->hp[i] = he[i] - ws->hdot * ws->nw[i];
            ws->tp[i] = te[i] - ws->tdot * ws->nw[i];
        }
        h = ws->hp;
        t = ws->tp;
    }
    if (norm_flag) {
        ws->hpn = normalize_into(h, ws->nh, d);
        ws->rn = normalize_into(re, ws->nr, d);
        ws->tpn = normalize_into(t, ws->nt, d);
    } else {
        memcpy(ws->nh, h, sizeof(float) * (size_t)d);
        memcpy(ws->nr, re, sizeof(float) * (size_t)d);
        memcpy(ws->nt, t, sizeof(float) * (size_t)d);
    }
    float s = 0;
    for (int64_t i = 0; i < d; ++i) {
        ws->v[i] = mode == 1 ? ws->nh[i] + (ws->nr[i] - ws->nt[i]) : (ws->nh[i] + ws->nr[i]) - ws->nt[i];
        s += p == 1 ? fabsf(ws->v[i]) : ws->v[i] * ws->v[i];
    }
    return p == 1 ? s : sqrtf(s);
}

void oracle_score(int model, int p, int norm_flag, int mode, int64_t d, const float *ent, const float *rel,
                  const float *normv, const int64_t *h, const int64_t *t, const int64_t *r, int64_t n, float *out) {
    float *buf = calloc((size_t)(11 * d), sizeof(float));
    slot_ws ws = {d, 0, 0, 0, 0, buf, buf + d, buf + 2 * d, buf + 3 * d, buf + 4 * d, buf + 5 * d, buf + 6 * d,
                  0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t i = 0; i < n; ++i)
        out[i] = slot_forward(model, p, norm_flag, mode, &ws, ent + h[i] * d, ent + t[i] * d, rel + r[i] * d,
                              model == 1 ? normv + r[i] * d : NULL);
    free(buf);
}

static void apply_update(int opt, float lr, float *w, float *acc, const float *g, int64_t n) {
    if (opt == 0) {
        for (int64_t i = 0; i < n; ++i) w[i] = w[i] + (-lr) * g[i];   /* SGD add_(grad, alpha=-lr) */
    } else {
        for (int64_t i = 0; i < n; ++i) {                               /* Adagrad, eps 1e-10, lr_decay 0 */
            acc[i] = acc[i] + g[i] * g[i];
            w[i] = w[i] + (-lr) * g[i] / (sqrtf(acc[i]) + 1e-10f);
        }
    }
}

/* ---------------------------------------------------------------- the step in reference order -- */
/* One step of Trainer.train_one_step (Trainer.py:44-56) in the order torch's autograd sums it:
 *   1. score every slot with the pre-step tables (TransE.py:46-74 / TransH.py:52-93);
 *   2. MarginLoss (MarginLoss.py:24-28) over NegativeSampling's (bs, neg) view (NegativeSampling.py:13-31):
 *      loss summed in (positive, negative) order, per-slot score gradients ds;
 *   3. per slot with ds != 0 its gradient rows: the h lookup's, the t lookup's, the r lookup's (and the
 *      norm_vector lookup's for TransH, the two _transfer calls' normalize backwards added, TransH.py:68-76);
 *   4. per table row the lookups' rows summed in slot order, each lookup separately, then the two entity
 *      lookups added (embedding_dense_backward per lookup, then AccumulateGrad, Trainer.py:52-55);
 *   5. the optimizer on every row with a gradient (a dense SGD / Adagrad step leaves the others unchanged).
 * Steps 1, 3 and 5 are independent per slot / per row; `workers` > 1 runs them on that many threads and
 * the result is bit-identical to workers = 1 (every float sum keeps its order). */
typedef struct {
    int model, p, norm_flag, opt;
    float lr, margin;
    int64_t E, R, d, bs, neg, seq;
    float *ent, *rel, *normv, *ent_acc, *rel_acc, *norm_acc;
    const int64_t *h, *t, *r;
    /* scratch */
    float *score, *ds;
    float *gh, *gt, *gr, *gw;                     /* [seq][d] */
    int64_t *hoff, *hlist, *toff, *tlist, *roff, *rlist;
    int64_t cap_seq, cap_e, cap_r, cap_d;
    /* oracle_grad_mass: per row element the summed gradient and the sum of its contributions' magnitudes
     * ([E + R (+ R)][d], entity rows then relation then norm_vector rows); the tables are not updated */
    float *gsum, *gmass;
} ostep;

static void slot_ws_bind(slot_ws *ws, float *buf, int64_t d) {
    memset(ws, 0, sizeof(*ws));
    ws->d = d;
    ws->hp = buf; ws->tp = buf + d; ws->nh = buf + 2 * d; ws->nt = buf + 3 * d; ws->nr = buf + 4 * d;
    ws->nw = buf + 5 * d; ws->v = buf + 6 * d;
}

/* d loss / d rows of slot s (step 3): writes gh/gt/gr(/gw) rows of the slot */
static void slot_backward(const ostep *S, slot_ws *ws, float *tmpb, int64_t s) {
    const int64_t d = S->d;
    const float *he = S->ent + S->h[s] * d, *te = S->ent + S->t[s] * d, *re = S->rel + S->r[s] * d;
    const float *W = S->model == 1 ? S->normv + S->r[s] * d : NULL;
    const float dsv = S->ds[s];
    float sc = slot_forward(S->model, S->p, S->norm_flag, 0, ws, he, te, re, W);
    float *gv = tmpb, *tmp = tmpb + d, *x1 = tmpb + 2 * d, *x2 = tmpb + 3 * d;
    float *ga = S->gh + s * d, *gb = S->gr + s * d, *gc = S->gt + s * d;
    for (int64_t i = 0; i < d; ++i) {
        if (S->p == 1) gv[i] = ws->v[i] > 0 ? dsv : (ws->v[i] < 0 ? -dsv : 0.0f);   /* sign(v), sign(0) = 0 */
        else gv[i] = sc == 0.0f ? 0.0f : ws->v[i] * (dsv / sc);
        tmp[i] = -gv[i];   /* d/d(nt) = -gv; d/d(nh) = d/d(nr) = gv */
    }
    const float *hsrc = S->model == 1 ? ws->hp : he, *tsrc = S->model == 1 ? ws->tp : te;
    if (S->norm_flag) {
        normalize_backward(hsrc, ws->hpn, gv, ga, d);
        normalize_backward(re, ws->rn, gv, gb, d);
        normalize_backward(tsrc, ws->tpn, tmp, gc, d);
    } else {
        memcpy(ga, gv, sizeof(float) * (size_t)d);
        memcpy(gb, gv, sizeof(float) * (size_t)d);
        memcpy(gc, tmp, sizeof(float) * (size_t)d);
    }
    if (S->model == 1) {
        /* e_perp = e - (e.n) n:  g_e = g_p - n (n.g_p);  g_n = -((e.n) g_p + (n.g_p) e), per _transfer call,
         * each through its own F.normalize(norm) backward */
        const float nga = vdot(ws->nw, ga, d), ngc = vdot(ws->nw, gc, d);
        for (int64_t i = 0; i < d; ++i) {
            tmp[i] = -(ws->hdot * ga[i] + nga * he[i]);
            gv[i] = -(ws->tdot * gc[i] + ngc * te[i]);
        }
        normalize_backward(W, ws->wn, tmp, x1, d);
        normalize_backward(W, ws->wn, gv, x2, d);
        float *gw = S->gw + s * d;
        for (int64_t i = 0; i < d; ++i) {
            gw[i] = x1[i] + x2[i];
            ga[i] = ga[i] - ws->nw[i] * nga;
            gc[i] = gc[i] - ws->nw[i] * ngc;
        }
    }
}

/* step 4 + 5 for one row: the listed slots' rows summed in slot order (per lookup), then the update */
static void row_update(const ostep *S, float *w, float *acc, const float *ga, const int64_t *la, int64_t na,
                       const float *gb, const int64_t *lb, int64_t nb, float *g) {
    /* per element: 0 + the lookup's rows in slot order (row by row over the list: the same per-element
     * order as element by element, with contiguous reads) */
    const int64_t d = S->d;
    float *b = g + d;
    memset(g, 0, sizeof(float) * (size_t)d);
    memset(b, 0, sizeof(float) * (size_t)d);
    for (int64_t k = 0; k < na; ++k) {
        const float *x = ga + la[k] * d;
        for (int64_t i = 0; i < d; ++i) g[i] += x[i];
    }
    for (int64_t k = 0; k < nb; ++k) {
        const float *x = gb + lb[k] * d;
        for (int64_t i = 0; i < d; ++i) b[i] += x[i];
    }
    if (nb)
        for (int64_t i = 0; i < d; ++i) g[i] = g[i] + b[i];
    apply_update(S->opt, S->lr, w, acc, g, d);
}

/* oracle_grad_mass's phase 2 for one row: the row gradient as row_update sums it, and sum |contribution| */
static void row_mass(const ostep *S, float *gs, float *gm, const float *ga, const int64_t *la, int64_t na,
                     const float *gb, const int64_t *lb, int64_t nb) {
    const int64_t d = S->d;
    for (int64_t i = 0; i < d; ++i) {
        float a = 0, b = 0, m = 0;
        for (int64_t k = 0; k < na; ++k) {
            const float x = ga[la[k] * d + i];
            a += x;
            m += fabsf(x);
        }
        for (int64_t k = 0; k < nb; ++k) {
            const float x = gb[lb[k] * d + i];
            b += x;
            m += fabsf(x);
        }
        gs[i] = nb ? a + b : a;
        gm[i] = m;
    }
}

/* counting sort of the slots with ds != 0 by key (stable: slots ascending inside a key) */
static void slot_csr(const ostep *S, const int64_t *key, int64_t nkeys, int64_t *off, int64_t *list) {
    memset(off, 0, sizeof(int64_t) * (size_t)(nkeys + 1));
    for (int64_t s = 0; s < S->seq; ++s)
        if (S->ds[s] != 0.0f) off[key[s] + 1] += 1;
    for (int64_t k = 0; k < nkeys; ++k) off[k + 1] += off[k];
    int64_t *cur = malloc(sizeof(int64_t) * (size_t)(nkeys ? nkeys : 1));
    memcpy(cur, off, sizeof(int64_t) * (size_t)nkeys);
    for (int64_t s = 0; s < S->seq; ++s)
        if (S->ds[s] != 0.0f) list[cur[key[s]]++] = s;
    free(cur);
}

typedef struct {
    const ostep *S;
    int phase;
    int64_t lo, hi;
} ojob;

static void run_range(const ostep *S, int phase, int64_t lo, int64_t hi) {
    const int64_t d = S->d;
    float *buf = calloc((size_t)(12 * d), sizeof(float));
    slot_ws ws;
    slot_ws_bind(&ws, buf, d);
    float *tmpb = buf + 7 * d;
    if (phase == 0) {
        for (int64_t s = lo; s < hi; ++s)
            S->score[s] = slot_forward(S->model, S->p, S->norm_flag, 0, &ws, S->ent + S->h[s] * d,
                                       S->ent + S->t[s] * d, S->rel + S->r[s] * d,
                                       S->model == 1 ? S->normv + S->r[s] * d : NULL);
    } else if (phase == 1) {
        for (int64_t s = lo; s < hi; ++s)
            if (S->ds[s] != 0.0f) slot_backward(S, &ws, tmpb, s);
    } else {
        /* rows: entities [0, E), relations [E, E + R), norm_vector rows [E + R, E + 2R) */
        for (int64_t q = lo; q < hi; ++q) {
            if (S->gsum) {   /* oracle_grad_mass: sums only */
                float *gs = S->gsum + q * d, *gm = S->gmass + q * d;
                if (q < S->E)
                    row_mass(S, gs, gm, S->gh, S->hlist + S->hoff[q], S->hoff[q + 1] - S->hoff[q], S->gt,
                             S->tlist + S->toff[q], S->toff[q + 1] - S->toff[q]);
                else {
                    const int64_t k = (q - S->E) % S->R;
                    row_mass(S, gs, gm, q < S->E + S->R ? S->gr : S->gw, S->rlist + S->roff[k],
                             S->roff[k + 1] - S->roff[k], NULL, NULL, 0);
                }
                continue;
            }
            if (q < S->E) {
                const int64_t na = S->hoff[q + 1] - S->hoff[q], nb = S->toff[q + 1] - S->toff[q];
                if (na + nb == 0) continue;
                /* the two lookups' dense gradients added: a row only one lookup touched is that lookup's sum */
                if (na)
                    row_update(S, S->ent + q * d, S->opt ? S->ent_acc + q * d : NULL, S->gh, S->hlist + S->hoff[q], na,
                               S->gt, S->tlist + S->toff[q], nb, tmpb);
                else
                    row_update(S, S->ent + q * d, S->opt ? S->ent_acc + q * d : NULL, S->gt, S->tlist + S->toff[q], nb,
                               S->gt, NULL, 0, tmpb);
            } else if (q < S->E + S->R) {
                const int64_t k = q - S->E, n = S->roff[k + 1] - S->roff[k];
                if (n)
                    row_update(S, S->rel + k * d, S->opt ? S->rel_acc + k * d : NULL, S->gr, S->rlist + S->roff[k], n,
                               S->gr, NULL, 0, tmpb);
            } else {
                const int64_t k = q - S->E - S->R, n = S->roff[k + 1] - S->roff[k];
                if (n)
                    row_update(S, S->normv + k * d, S->opt ? S->norm_acc + k * d : NULL, S->gw, S->rlist + S->roff[k],
                               n, S->gw, NULL, 0, tmpb);
            }
        }
    }
    free(buf);
}

static void *run_job(void *arg) {
    const ojob *j = (const ojob *)arg;
    run_range(j->S, j->phase, j->lo, j->hi);
    return NULL;
}

static void parallel_phase(const ostep *S, int phase, int64_t n, int64_t workers) {
    if (workers <= 1 || n < 2 * workers) {
        run_range(S, phase, 0, n);
        return;
    }
    pthread_t th[256];
    ojob jobs[256];
    if (workers > 256) workers = 256;
    for (int64_t w = 0; w < workers; ++w) {
        jobs[w].S = S;
        jobs[w].phase = phase;
        jobs[w].lo = n * w / workers;
        jobs[w].hi = n * (w + 1) / workers;
        pthread_create(&th[w], NULL, run_job, &jobs[w]);
    }
    for (int64_t w = 0; w < workers; ++w) pthread_join(th[w], NULL);
}

static void ostep_reserve(ostep *S) {
    const int64_t seq = S->seq, d = S->d;
    if (seq > S->cap_seq || d != S->cap_d) {
        free(S->score); free(S->ds); free(S->gh); free(S->gt); free(S->gr); free(S->gw);
        free(S->hlist); free(S->tlist); free(S->rlist);
        S->score = malloc(sizeof(float) * (size_t)seq);
        S->ds = malloc(sizeof(float) * (size_t)seq);
        S->gh = malloc(sizeof(float) * (size_t)(seq * d));
        S->gt = malloc(sizeof(float) * (size_t)(seq * d));
        S->gr = malloc(sizeof(float) * (size_t)(seq * d));
        S->gw = malloc(sizeof(float) * (size_t)(seq * d));
        S->hlist = malloc(sizeof(int64_t) * (size_t)seq);
        S->tlist = malloc(sizeof(int64_t) * (size_t)seq);
        S->rlist = malloc(sizeof(int64_t) * (size_t)seq);
        S->cap_seq = seq;
        S->cap_d = d;
    }
    if (S->E > S->cap_e) {
        free(S->hoff); free(S->toff);
        S->hoff = malloc(sizeof(int64_t) * (size_t)(S->E + 1));
        S->toff = malloc(sizeof(int64_t) * (size_t)(S->E + 1));
        S->cap_e = S->E;
    }
    if (S->R > S->cap_r) {
        free(S->roff);
        S->roff = malloc(sizeof(int64_t) * (size_t)(S->R + 1));
        S->cap_r = S->R;
    }
}

static void ostep_release(ostep *S) {
    free(S->score); free(S->ds); free(S->gh); free(S->gt); free(S->gr); free(S->gw);
    free(S->hlist); free(S->tlist); free(S->rlist); free(S->hoff); free(S->toff); free(S->roff);
}

static float ostep_run(ostep *S, int64_t workers) {
    ostep_reserve(S);
    const int64_t bs = S->bs, neg = S->neg, seq = S->seq;
    parallel_phase(S, 0, seq, workers);
    /* MarginLoss: mean(max(p - n, -m)) + m; NegativeSampling reshape n[i][k] = score[bs + k*bs + i] */
    double lsum = 0;
    const float inv = 1.0f / (float)(bs * neg), margin = S->margin;
    memset(S->ds, 0, sizeof(float) * (size_t)seq);
    for (int64_t i = 0; i < bs; ++i)
        for (int64_t k = 0; k < neg; ++k) {
            const float a = S->score[i] - S->score[bs + k * bs + i];
            const float mx = a > -margin ? a : -margin;
            lsum += mx;
            const float c = a > -margin ? inv : (a == -margin ? inv / 2 : 0.0f);
            S->ds[i] += c;
            S->ds[bs + k * bs + i] -= c;
        }
    const float loss = (float)(lsum / (double)(bs * neg)) + margin;
    parallel_phase(S, 1, seq, workers);
    slot_csr(S, S->h, S->E, S->hoff, S->hlist);
    slot_csr(S, S->t, S->E, S->toff, S->tlist);
    slot_csr(S, S->r, S->R, S->roff, S->rlist);
    parallel_phase(S, 2, S->E + S->R * (S->model == 1 ? 2 : 1), workers);
    return loss;
}

float oracle_train_step(int model, int p, int norm_flag, int opt, float lr, float margin, int64_t E, int64_t R,
                        int64_t d, float *ent, float *rel, float *normv, float *ent_acc, float *rel_acc,
                        float *norm_acc, const int64_t *h, const int64_t *t, const int64_t *r, int64_t bs,
                        int64_t neg) {
    return oracle_train_step_mt(model, p, norm_flag, opt, lr, margin, E, R, d, ent, rel, normv, ent_acc, rel_acc,
                                norm_acc, h, t, r, bs, neg, 1);
}

float oracle_train_step_mt(int model, int p, int norm_flag, int opt, float lr, float margin, int64_t E, int64_t R,
                           int64_t d, float *ent, float *rel, float *normv, float *ent_acc, float *rel_acc,
                           float *norm_acc, const int64_t *h, const int64_t *t, const int64_t *r, int64_t bs,
                           int64_t neg, int64_t workers) {
    ostep S;
    memset(&S, 0, sizeof(S));
    S.model = model; S.p = p; S.norm_flag = norm_flag; S.opt = opt; S.lr = lr; S.margin = margin;
    S.E = E; S.R = R; S.d = d; S.bs = bs; S.neg = neg; S.seq = bs * (1 + neg);
    S.ent = ent; S.rel = rel; S.normv = normv; S.ent_acc = ent_acc; S.rel_acc = rel_acc; S.norm_acc = norm_acc;
    S.h = h; S.t = t; S.r = r;
    const float loss = ostep_run(&S, workers);
    ostep_release(&S);
    return loss;
}

/* Test infrastructure for the fast kernels' step tolerance (tests/helpers.py kappa_bound): at the given tables
 * and batch, without updating anything, per table element
 *   gsum  - the step's gradient, summed in the reference's order (row_update);
 *   gmass - the sum of its per-slot contributions' magnitudes;
 *   gabs  - the same gradient evaluated with absolute values throughout (|.| of every operand of the forward
 *           pieces a contribution depends on, the normalize / projection Jacobians with |x| and sums of
 *           magnitudes): standard forward-error analysis bounds the rounding error of ANY evaluation order of the
 *           gradient by k * eps * gabs, k the length of the longest chain of operations;
 * per row
 *   gcnt  - contributions (slots with a nonzero score gradient touching the row);
 *   gtie  - 1 when a slot touching the row had a near-tie decision: a margin comparison p - n vs -m, or (p = 1)
 *           a sign(v_i), within rounding of its threshold. There two correct float32 implementations may take
 *           different branches (a discrete difference no eps bound covers), so the tests exempt those rows.
 * Outputs [E + R (+ R for TransH)][d] (entity, relation, norm_vector rows) and [E + R (+ R)]. Returns the loss. */
static void nb_abs(const float *x, float n, const float *g, float *out, int64_t d) {
    if (n > 1e-12f) {
        float c = 0;
        for (int64_t i = 0; i < d; ++i) c += fabsf(x[i]) * g[i];
        c /= n * n;
        for (int64_t i = 0; i < d; ++i) out[i] = (g[i] + fabsf(x[i]) * c) / n;
    } else {
        for (int64_t i = 0; i < d; ++i) out[i] = g[i] / 1e-12f;
    }
}

float oracle_grad_mass(int model, int p, int norm_flag, float margin, int64_t E, int64_t R, int64_t d, float *ent,
                       float *rel, float *normv, const int64_t *h, const int64_t *t, const int64_t *r, int64_t bs,
                       int64_t neg, float *gsum, float *gmass, float *gabs, int32_t *gcnt, int32_t *gtie) {
    ostep S;
    memset(&S, 0, sizeof(S));
    S.model = model; S.p = p; S.norm_flag = norm_flag; S.opt = 0; S.lr = 0.f; S.margin = margin;
    S.E = E; S.R = R; S.d = d; S.bs = bs; S.neg = neg; S.seq = bs * (1 + neg);
    S.ent = ent; S.rel = rel; S.normv = normv;
    S.h = h; S.t = t; S.r = r;
    S.gsum = gsum;
    S.gmass = gmass;
    const float loss = ostep_run(&S, 1);   /* scores, ds, per-slot rows, gsum / gmass */
    const int64_t seq = S.seq, rows = E + R * (model == 1 ? 2 : 1);
    const float eps = 5.9604645e-8f;   /* 2^-24 */
    memset(gabs, 0, sizeof(float) * (size_t)(rows * d));
    memset(gcnt, 0, sizeof(int32_t) * (size_t)rows);
    memset(gtie, 0, sizeof(int32_t) * (size_t)rows);
    float *buf = calloc((size_t)(20 * d), sizeof(float));
    float *sabs = calloc((size_t)seq, sizeof(float));
    int8_t *tie = calloc((size_t)seq, 1);
    slot_ws ws;
    slot_ws_bind(&ws, buf, d);
    float *gv = buf + 7 * d, *ga = buf + 8 * d, *gb = buf + 9 * d, *gc = buf + 10 * d, *gw = buf + 11 * d;
    float *x1 = buf + 12 * d, *x2 = buf + 13 * d, *t1 = buf + 14 * d, *t2 = buf + 15 * d;
    /* absolute evaluation of every score (the terms of v) and the sign near-ties (p = 1) */
    for (int64_t s = 0; s < seq; ++s) {
        slot_forward(model, p, norm_flag, 0, &ws, ent + h[s] * d, ent + t[s] * d, rel + r[s] * d,
                     model == 1 ? normv + r[s] * d : NULL);
        float a = 0;
        for (int64_t i = 0; i < d; ++i) {
            const float m = fabsf(ws.nh[i]) + fabsf(ws.nr[i]) + fabsf(ws.nt[i]);
            a += m;
            if (p == 1 && fabsf(ws.v[i]) <= 2.f * (float)(d + 8) * eps * m) tie[s] = 1;
        }
        sabs[s] = a;
    }
    /* margin near-ties: p - n within rounding of -m (MarginLoss.py:24-28) */
    for (int64_t i = 0; i < bs; ++i)
        for (int64_t k = 0; k < neg; ++k) {
            const int64_t q = bs + k * bs + i;
            const float a = S.score[i] - S.score[q];
            if (fabsf(a + margin) <= 2.f * (float)(d + 16) * eps * (sabs[i] + sabs[q])) tie[i] = tie[q] = 1;
        }
    for (int64_t s = 0; s < seq; ++s) {
        const int64_t rh = h[s], rt = t[s], rr = E + r[s], rw = E + R + r[s];
        if (tie[s]) {
            gtie[rh] = gtie[rt] = gtie[rr] = 1;
            if (model == 1) gtie[rw] = 1;
        }
        if (S.ds[s] == 0.0f) continue;
        const float *he = ent + h[s] * d, *te = ent + t[s] * d, *re = rel + r[s] * d;
        const float *W = model == 1 ? normv + r[s] * d : NULL;
        const float sc = slot_forward(model, p, norm_flag, 0, &ws, he, te, re, W);
        const float ads = fabsf(S.ds[s]);
        for (int64_t i = 0; i < d; ++i)
            gv[i] = p == 1 ? ads : (sc == 0.0f ? 0.0f : ads / sc * (fabsf(ws.v[i]) + fabsf(ws.nh[i]) +
                                                                       fabsf(ws.nr[i]) + fabsf(ws.nt[i])));
        const float *hsrc = model == 1 ? ws.hp : he, *tsrc = model == 1 ? ws.tp : te;
        if (norm_flag) {
            nb_abs(hsrc, ws.hpn, gv, ga, d);
            nb_abs(re, ws.rn, gv, gb, d);
            nb_abs(tsrc, ws.tpn, gv, gc, d);
        } else {
            memcpy(ga, gv, sizeof(float) * (size_t)d);
            memcpy(gb, gv, sizeof(float) * (size_t)d);
            memcpy(gc, gv, sizeof(float) * (size_t)d);
        }
        if (model == 1) {   /* the projection's Jacobians (TransH.py:68-76) with magnitudes */
            float nga = 0, ngc = 0, hd = 0, td = 0;
            for (int64_t i = 0; i < d; ++i) {
                nga += fabsf(ws.nw[i]) * ga[i];
                ngc += fabsf(ws.nw[i]) * gc[i];
                hd += fabsf(he[i]) * fabsf(ws.nw[i]);
                td += fabsf(te[i]) * fabsf(ws.nw[i]);
            }
            for (int64_t i = 0; i < d; ++i) {
                t1[i] = hd * ga[i] + nga * fabsf(he[i]);
                t2[i] = td * gc[i] + ngc * fabsf(te[i]);
            }
            nb_abs(W, ws.wn, t1, x1, d);
            nb_abs(W, ws.wn, t2, x2, d);
            for (int64_t i = 0; i < d; ++i) {
                gw[i] = x1[i] + x2[i];
                ga[i] = ga[i] + fabsf(ws.nw[i]) * nga;
                gc[i] = gc[i] + fabsf(ws.nw[i]) * ngc;
            }
        }
        float *ah = gabs + rh * d, *at = gabs + rt * d, *ar = gabs + rr * d;
        for (int64_t i = 0; i < d; ++i) {
            ah[i] += ga[i];
            at[i] += gc[i];
            ar[i] += gb[i];
        }
        gcnt[rh] += 1;
        gcnt[rt] += 1;
        gcnt[rr] += 1;
        if (model == 1) {
            float *aw = gabs + rw * d;
            for (int64_t i = 0; i < d; ++i) aw[i] += gw[i];
            gcnt[rw] += 1;
        }
    }
    free(buf);
    free(sabs);
    free(tie);
    ostep_release(&S);
    return loss;
}

/* the sampler threads' slices of one sampling() call on `workers` threads (each slice owns its stream,
 * Base.cpp:280-298, so the batch is the same as oracle_sampling's) */
typedef struct {
    const okg *g;
    uint64_t *states;
    int64_t threads, bs, neg, bern, filter, id0, id1;
    int64_t *h, *t, *r;
    float *y;
} osamp;

static void *samp_job(void *arg) {
    const osamp *a = (const osamp *)arg;
    for (int64_t id = a->id0; id < a->id1; ++id) {
        /* one sampler thread = oracle_sampling_sides restricted to thread id's slice */
        int64_t lef, rig;
        if (a->bs % a->threads == 0) {
            lef = id * (a->bs / a->threads);
            rig = (id + 1) * (a->bs / a->threads);
        } else {
            lef = id * (a->bs / a->threads + 1);
            rig = (id + 1) * (a->bs / a->threads + 1);
            if (rig > a->bs) rig = a->bs;
        }
        if (lef >= rig) continue;
        uint64_t *s = &a->states[id];
        const okg *g = a->g;
        float prob = 500;
        for (int64_t b = lef; b < rig; ++b) {
            int64_t i = lcg_max(s, g->train_total);
            otriple pp = g->train_list[i];
            a->h[b] = pp.h; a->t[b] = pp.t; a->r[b] = pp.r; a->y[b] = 1;
            int64_t last = a->bs;
            for (int64_t k = 0; k < a->neg; ++k) {
                if (a->bern) prob = 1000 * g->right_mean[pp.r] / (g->right_mean[pp.r] + g->left_mean[pp.r]);
                if ((float)(lcg_next(s) % 1000) < prob) {
                    a->h[b + last] = pp.h;
                    a->t[b + last] = a->filter ? corrupt_filtered(g, 1, pp.h, pp.r, s) : corrupt_plain(g, pp.h, s);
                } else {
                    a->h[b + last] = a->filter ? corrupt_filtered(g, 0, pp.t, pp.r, s) : corrupt_plain(g, pp.t, s);
                    a->t[b + last] = pp.t;
                }
                a->r[b + last] = pp.r;
                a->y[b + last] = -1;
                last += a->bs;
            }
        }
    }
    return NULL;
}

static void sampling_mt(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t bern,
                        int64_t filter, int64_t *h, int64_t *t, int64_t *r, float *y, int64_t workers) {
    if (workers > threads) workers = threads;
    if (workers <= 1) {
        oracle_sampling(g, states, threads, bs, neg, bern, filter, h, t, r, y);
        return;
    }
    pthread_t th[64];
    osamp a[64];
    for (int64_t w = 0; w < workers; ++w) {
        a[w] = (osamp){g, states, threads, bs, neg, bern, filter, threads * w / workers, threads * (w + 1) / workers,
                       h, t, r, y};
        pthread_create(&th[w], NULL, samp_job, &a[w]);
    }
    for (int64_t w = 0; w < workers; ++w) pthread_join(th[w], NULL);
}

int64_t oracle_train_loop_mt(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t bern,
                             int64_t filter, int model, int p, int norm_flag, int opt, float lr, float margin,
                             int64_t d, float *ent, float *rel, float *normv, float *ent_acc, float *rel_acc,
                             float *norm_acc, int64_t steps, int64_t workers, float *losses) {
    int64_t seq = bs * (1 + neg);
    int64_t *h = malloc(sizeof(int64_t) * (size_t)seq), *t = malloc(sizeof(int64_t) * (size_t)seq);
    int64_t *r = malloc(sizeof(int64_t) * (size_t)seq);
    float *y = malloc(sizeof(float) * (size_t)seq);
    ostep S;
    memset(&S, 0, sizeof(S));
    S.model = model; S.p = p; S.norm_flag = norm_flag; S.opt = opt; S.lr = lr; S.margin = margin;
    S.E = g->ent_total; S.R = g->rel_total; S.d = d; S.bs = bs; S.neg = neg; S.seq = seq;
    S.ent = ent; S.rel = rel; S.normv = normv; S.ent_acc = ent_acc; S.rel_acc = rel_acc; S.norm_acc = norm_acc;
    S.h = h; S.t = t; S.r = r;
    for (int64_t s = 0; s < steps; ++s) {
        sampling_mt(g, states, threads, bs, neg, bern, filter, h, t, r, y, workers);
        const float l = ostep_run(&S, workers);
        if (losses) losses[s] = l;
    }
    ostep_release(&S);
    free(h); free(t); free(r); free(y);
    return steps * seq;
}

int64_t oracle_train_loop(const okg *g, uint64_t *states, int64_t threads, int64_t bs, int64_t neg, int64_t bern,
                          int64_t filter, int model, int p, int norm_flag, int opt, float lr, float margin, int64_t d,
                          float *ent, float *rel, float *normv, float *ent_acc, float *rel_acc, float *norm_acc,
                          int64_t steps) {
    return oracle_train_loop_mt(g, states, threads, bs, neg, bern, filter, model, p, norm_flag, opt, lr, margin, d,
                                ent, rel, normv, ent_acc, rel_acc, norm_acc, steps, 1, NULL);
}

/* ---------------------------------------------------------------- link prediction ------------- */
void oracle_sort_test(int64_t n, int64_t *h, int64_t *t, int64_t *r) {   /* importTestFiles :311 */
    otriple *a = malloc(sizeof(otriple) * (size_t)(n ? n : 1));
    for (int64_t i = 0; i < n; ++i) { a[i].h = h[i]; a[i].t = t[i]; a[i].r = r[i]; }
    qsort(a, (size_t)n, sizeof(otriple), cmp_rel2);
    for (int64_t i = 0; i < n; ++i) { h[i] = a[i].h; t[i] = a[i].t; r[i] = a[i].r; }
    free(a);
}

static int find_triple(const otriple *all, int64_t n, int64_t h, int64_t t, int64_t r) {   /* _find */
    otriple key = {h, r, t};
    return bsearch(&key, all, (size_t)n, sizeof(otriple), cmp_head) != NULL;
}

/* filtered MRR / MR / Hits@10/3/1 from the per-query filtered ranks, with the reference's float
 * accumulators per side (Test.h:213-223, :333-343, :398-454) */
void oracle_metrics_from_ranks(int64_t n_test, const int64_t *frank_head, const int64_t *frank_tail, float *metrics) {
    float l_filter_tot = 0, l3_filter_tot = 0, l1_filter_tot = 0, l_filter_rank = 0, l_filter_reci = 0;
    float r_filter_tot = 0, r3_filter_tot = 0, r1_filter_tot = 0, r_filter_rank = 0, r_filter_reci = 0;
    for (int64_t q = 0; q < n_test; ++q) {
        const int64_t fh = frank_head[q], ft = frank_tail[q];
        if (fh < 10) l_filter_tot += 1;
        if (fh < 3) l3_filter_tot += 1;
        if (fh < 1) l1_filter_tot += 1;
        l_filter_rank += (float)(fh + 1);
        l_filter_reci = (float)((double)l_filter_reci + 1.0 / (double)(fh + 1));
        if (ft < 10) r_filter_tot += 1;
        if (ft < 3) r3_filter_tot += 1;
        if (ft < 1) r1_filter_tot += 1;
        r_filter_rank += (float)(1 + ft);
        r_filter_reci = (float)((double)r_filter_reci + 1.0 / (double)(1 + ft));
    }
    float nt = (float)n_test;
    l_filter_rank /= nt; r_filter_rank /= nt; l_filter_reci /= nt; r_filter_reci /= nt;
    l_filter_tot /= nt; l3_filter_tot /= nt; l1_filter_tot /= nt;
    r_filter_tot /= nt; r3_filter_tot /= nt; r1_filter_tot /= nt;
    metrics[0] = (l_filter_reci + r_filter_reci) / 2;       /* Test.h:450-454 */
    metrics[1] = (l_filter_rank + r_filter_rank) / 2;
    metrics[2] = (l_filter_tot + r_filter_tot) / 2;
    metrics[3] = (l3_filter_tot + r3_filter_tot) / 2;
    metrics[4] = (l1_filter_tot + r1_filter_tot) / 2;
}

void oracle_link_prediction(int64_t E, const int64_t *ah, const int64_t *at, const int64_t *ar, int64_t n_all,
                            const int64_t *th, const int64_t *tt, const int64_t *tr, int64_t n_test,
                            const float *con_head, const float *con_tail, int64_t *rank_head, int64_t *frank_head,
                            int64_t *rank_tail, int64_t *frank_tail, float *metrics) {
    otriple *all = malloc(sizeof(otriple) * (size_t)(n_all ? n_all : 1));
    for (int64_t i = 0; i < n_all; ++i) { all[i].h = ah[i]; all[i].t = at[i]; all[i].r = ar[i]; }
    qsort(all, (size_t)n_all, sizeof(otriple), cmp_head);
    for (int64_t q = 0; q < n_test; ++q) {
        int64_t h = th[q], t = tt[q], r = tr[q];
        for (int side = 0; side < 2; ++side) {     /* 0: testHead (Test.h:118-238), 1: testTail (:240-359) */
            const float *con = (side == 0 ? con_head : con_tail) + q * E;
            int64_t truth = side == 0 ? h : t;
            int64_t raw = 0, filt = 0;
            float minimal = con[0];
            if (minimal != INFINITY) {
                for (int64_t j = 1; j < E; ++j) {
                    int64_t cand = j - 1 < truth ? j - 1 : j;
                    if (con[j] < minimal) {
                        raw++;
                        int known = side == 0 ? find_triple(all, n_all, cand, t, r) : find_triple(all, n_all, h, cand, r);
                        if (!known) filt++;
                    }
                }
            } else {
                raw = E;
                filt = E;
                for (int64_t j = 1; j < E; ++j) {
                    int64_t cand = j - 1 < truth ? j - 1 : j;
                    int known = side == 0 ? find_triple(all, n_all, cand, t, r) : find_triple(all, n_all, h, cand, r);
                    if (known) filt--;
                }
            }
            if (side == 0) {
                rank_head[q] = raw; frank_head[q] = filt;
            } else {
                rank_tail[q] = raw; frank_tail[q] = filt;
            }
        }
    }
    oracle_metrics_from_ranks(n_test, frank_head, frank_tail, metrics);
    free(all);
}

/* Type-constrained counts of testHead / testTail (Test.h:127-130, :168-178, :225-237 and the tail mirror
 * :248-251, :288-298, :346-358), restated literally: j walks the candidate POSITIONS 1..E-1 while the
 * sorted type list of r is scanned for j as an ENTITY id, so con[j] (the score of the candidate at
 * position j) is compared for entity j, and the filter asks _find for entity j. Nothing is counted when
 * con[0] == inf. Metrics as the constrained block of test_link_prediction (Test.h:456-502). */
void oracle_rank_constrained(int64_t E, const int64_t *ah, const int64_t *at, const int64_t *ar, int64_t n_all,
                             const int64_t *th, const int64_t *tt, const int64_t *tr, int64_t n_test,
                             const float *con_head, const float *con_tail, const int64_t *head_lef,
                             const int64_t *head_rig, const int64_t *head_type, const int64_t *tail_lef,
                             const int64_t *tail_rig, const int64_t *tail_type, int64_t *rank_head,
                             int64_t *frank_head, int64_t *rank_tail, int64_t *frank_tail, float *metrics) {
    otriple *all = malloc(sizeof(otriple) * (size_t)(n_all ? n_all : 1));
    for (int64_t i = 0; i < n_all; ++i) { all[i].h = ah[i]; all[i].t = at[i]; all[i].r = ar[i]; }
    qsort(all, (size_t)n_all, sizeof(otriple), cmp_head);
    float lt = 0, l3 = 0, l1 = 0, lr = 0, li = 0, rt = 0, r3 = 0, r1 = 0, rr_ = 0, ri = 0;
    for (int64_t q = 0; q < n_test; ++q) {
        int64_t h = th[q], t = tt[q], r = tr[q];
        for (int side = 0; side < 2; ++side) {
            const float *con = (side == 0 ? con_head : con_tail) + q * E;
            const int64_t *type = side == 0 ? head_type : tail_type;
            int64_t lef = side == 0 ? head_lef[r] : tail_lef[r], rig = side == 0 ? head_rig[r] : tail_rig[r];
            int64_t s = 0, fs = 0;
            const float minimal = con[0];
            if (minimal != INFINITY) {
                for (int64_t j = 1; j < E; ++j) {
                    while (lef < rig && type[lef] < j) lef++;
                    if (lef < rig && j == type[lef] && con[j] < minimal) {
                        s++;
                        int known = side == 0 ? find_triple(all, n_all, j, t, r) : find_triple(all, n_all, h, j, r);
                        if (!known) fs++;
                    }
                }
            }
            if (side == 0) {
                rank_head[q] = s; frank_head[q] = fs;
                if (fs < 10) lt += 1;
                if (fs < 3) l3 += 1;
                if (fs < 1) l1 += 1;
                lr += (float)(fs + 1);
                li = (float)((double)li + 1.0 / (double)(fs + 1));
            } else {
                rank_tail[q] = s; frank_tail[q] = fs;
                if (fs < 10) rt += 1;
                if (fs < 3) r3 += 1;
                if (fs < 1) r1 += 1;
                rr_ += (float)(1 + fs);
                ri = (float)((double)ri + 1.0 / (double)(1 + fs));
            }
        }
    }
    float nt = (float)n_test;
    lr /= nt; rr_ /= nt; li /= nt; ri /= nt;
    lt /= nt; l3 /= nt; l1 /= nt;
    rt /= nt; r3 /= nt; r1 /= nt;
    metrics[0] = (li + ri) / 2;                             /* Test.h:498-502 */
    metrics[1] = (lr + rr_) / 2;
    metrics[2] = (lt + rt) / 2;
    metrics[3] = (l3 + r3) / 2;
    metrics[4] = (l1 + r1) / 2;
    free(all);
}
