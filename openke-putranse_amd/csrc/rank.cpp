// Link-prediction ranking (testHead / testTail, Test.h:118-359) over many queries on host threads,
// with the known-triple filter (_find over tripleList, Corrupt.h:188-199) as a hash set.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "common.h"

namespace {
inline uint64_t pack(int64_t h, int64_t t, int64_t r) {
    return ((uint64_t)h * 0x9E3779B97F4A7C15ULL) ^ ((uint64_t)t * 0xC2B2AE3D27D4EB4FULL) ^ ((uint64_t)r << 1);
}
struct Key {
    int64_t h, t, r;
    bool operator==(const Key &o) const { return h == o.h && t == o.t && r == o.r; }
};
struct KeyHash {
    size_t operator()(const Key &k) const {
        uint64_t x = pack(k.h, k.t, k.r);
        return (size_t)(x ^ (x >> 31));
    }
};
}  // namespace

struct pt_known {
    std::unordered_set<Key, KeyHash> set;
    std::vector<Key> triples;   // as given (duplicates included): the partner index is sorted from these
    bool has(int64_t h, int64_t t, int64_t r) const { return set.count(Key{h, t, r}) != 0; }
    // (anchor, r, partner) rows per side (0: heads of (t, r); 1: tails of (h, r)), sorted, so a query's partners
    // are one contiguous ascending run found by bisection; built on first use, the two sides on two threads (a
    // sort of the known triples instead of a hash map of vectors: C4's 318 k triples)
    struct Row {
        int64_t a, r, p;
        bool operator<(const Row &o) const { return a != o.a ? a < o.a : r != o.r ? r < o.r : p < o.p; }
    };
    mutable std::mutex mu;
    mutable bool indexed = false;
    mutable std::vector<Row> by_side[2];
    void index() const {
        std::lock_guard<std::mutex> g(mu);
        if (indexed) return;
        auto build = [this](int side) {
            // a counting sort by anchor, then each anchor's few rows sorted by (r, partner)
            auto &v = by_side[side];
            int64_t amax = -1, amin = 0;
            for (const Key &k : triples) {
                amax = std::max(amax, side == 0 ? k.t : k.h);
                amin = std::min(amin, side == 0 ? k.t : k.h);
            }
            if (amin < 0 || amax >= (int64_t(1) << 32)) {   // (ids a counting sort cannot index: a plain sort)
                for (const Key &k : triples) v.push_back(side == 0 ? Row{k.t, k.r, k.h} : Row{k.h, k.r, k.t});
                std::sort(v.begin(), v.end());
                v.erase(std::unique(v.begin(), v.end(), [](const Row &x, const Row &y) {
                            return x.a == y.a && x.r == y.r && x.p == y.p;
                        }),
                        v.end());
                return;
            }
            std::vector<int64_t> start((size_t)(amax + 2), 0);
            for (const Key &k : triples) ++start[(size_t)((side == 0 ? k.t : k.h) + 1)];
            for (size_t a = 1; a < start.size(); ++a) start[a] += start[a - 1];
            v.resize(triples.size());
            {
                std::vector<int64_t> fill(start.begin(), start.end() - 1);
                for (const Key &k : triples)
                    v[(size_t)fill[(size_t)(side == 0 ? k.t : k.h)]++] =
                        side == 0 ? Row{k.t, k.r, k.h} : Row{k.h, k.r, k.t};
            }
            for (size_t a = 0; a + 1 < start.size(); ++a)
                if (start[a + 1] - start[a] > 1) std::sort(v.begin() + start[a], v.begin() + start[a + 1]);
            v.erase(std::unique(v.begin(), v.end(), [](const Row &x, const Row &y) {
                        return x.a == y.a && x.r == y.r && x.p == y.p;
                    }),
                    v.end());   // (a triple listed twice is one known triple)
        };
        std::thread other(build, 1);
        build(0);
        other.join();
        indexed = true;
    }
    // the run of (a, r)'s partners in side `side`'s rows
    std::pair<const Row *, const Row *> partners(int side, int64_t a, int64_t r) const {
        const auto &v = by_side[side];
        const auto lo = std::lower_bound(v.begin(), v.end(), Row{a, r, INT64_MIN});
        auto hi = lo;
        while (hi != v.end() && hi->a == a && hi->r == r) ++hi;
        return {v.data() + (lo - v.begin()), v.data() + (hi - v.begin())};
    }
};

namespace pt {
// rank of one query: raw = #{j>=1: con[j] < con[0]}; filtered drops known triples; con[0] == inf
// ranks last (entity_total minus the known candidates), exactly as Test.h:138-207.
void rank_one(const pt_known &k, int64_t E, int64_t h, int64_t t, int64_t r, int side, const float *con,
              int64_t *raw, int64_t *filt) {
    const int64_t truth = side == 0 ? h : t;
    const float minimal = con[0];
    int64_t rs = 0, fs = 0;
    if (minimal != INFINITY) {
        for (int64_t j = 1; j < E; ++j) {
            if (con[j] < minimal) {
                const int64_t cand = j - 1 < truth ? j - 1 : j;
                ++rs;
                if (!(side == 0 ? k.has(cand, t, r) : k.has(h, cand, r))) ++fs;
            }
        }
    } else {
        rs = fs = E;
        for (int64_t j = 1; j < E; ++j) {
            const int64_t cand = j - 1 < truth ? j - 1 : j;
            if (side == 0 ? k.has(cand, t, r) : k.has(h, cand, r)) --fs;
        }
    }
    *raw = rs;
    *filt = fs;
}
bool known_has(const pt_known &k, int64_t h, int64_t t, int64_t r) { return k.has(h, t, r); }
}  // namespace pt

extern "C" int pt_known_create(const int64_t *h, const int64_t *t, const int64_t *r, int64_t n, pt_known **out) {
    if (!out || (n > 0 && (!h || !t || !r))) return pt::fail(PT_EINVAL, "pt_known_create: null argument");
    auto *k = new pt_known();
    k->set.reserve((size_t)n * 2 + 16);
    k->triples.resize((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        k->triples[(size_t)i] = Key{h[i], t[i], r[i]};
        k->set.insert(k->triples[(size_t)i]);
    }
    *out = k;
    return PT_OK;
}

extern "C" int pt_known_free(pt_known *k) {
    delete k;
    return PT_OK;
}

extern "C" int pt_rank_queries(const pt_known *k, int64_t E, const int64_t *h, const int64_t *t, const int64_t *r,
                               int64_t n, int32_t side, const float *con, int64_t *raw, int64_t *filt,
                               int64_t n_workers) {
    if (!k || (n > 0 && (!h || !t || !r || !con || !raw || !filt)))
        return pt::fail(PT_EINVAL, "pt_rank_queries: null argument");
    if (n_workers <= 0) n_workers = std::max(1u, std::thread::hardware_concurrency());
    n_workers = std::min<int64_t>(n_workers, std::max<int64_t>(n, 1));
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        for (int64_t q; (q = next.fetch_add(1)) < n;)
            pt::rank_one(*k, E, h[q], t[q], r[q], side, con + q * E, raw + q, filt + q);
    };
    std::vector<std::thread> pool;
    for (int64_t w = 1; w < n_workers; ++w) pool.emplace_back(work);
    work();
    for (auto &th : pool) th.join();
    return PT_OK;
}

// CSR of the known partners of many (anchor, r) queries: side 0 (head prediction, anchor = t) lists the
// h with (h, t, r) known; side 1 (tail prediction, anchor = h) lists the t with (h, t, r) known.
// off[n + 1]; when list is NULL only off is filled (off[n] = total). Each query's list is ascending.
extern "C" int pt_known_partners(const pt_known *k, int32_t side, int64_t n, const int64_t *anchor, const int64_t *rel,
                                 int64_t *off, int64_t *list) {
    if (!k || (n > 0 && (!anchor || !rel)) || !off || (side != 0 && side != 1))
        return pt::fail(PT_EINVAL, "pt_known_partners: bad argument");
    k->index();
    off[0] = 0;
    for (int64_t q = 0; q < n; ++q) {
        const auto run = k->partners(side, anchor[q], rel[q]);   // ascending: pt_rank_types bisects it
        const int64_t c = run.second - run.first;
        if (list)
            for (int64_t i = 0; i < c; ++i) list[off[q] + i] = run.first[i].p;
        off[q + 1] = off[q] + c;
    }
    return PT_OK;
}
