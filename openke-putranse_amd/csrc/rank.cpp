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
    bool has(int64_t h, int64_t t, int64_t r) const { return set.count(Key{h, t, r}) != 0; }
    // (anchor, r) -> partner entities, per side (0: heads of (t, r); 1: tails of (h, r)); built on first use
    struct PairHash {
        size_t operator()(const std::pair<int64_t, int64_t> &p) const {
            const uint64_t x = (uint64_t)p.first * 0x9E3779B97F4A7C15ULL ^ (uint64_t)p.second * 0xC2B2AE3D27D4EB4FULL;
            return (size_t)(x ^ (x >> 29));
        }
    };
    mutable std::mutex mu;
    mutable bool indexed = false;
    mutable std::unordered_map<std::pair<int64_t, int64_t>, std::vector<int64_t>, PairHash> by_side[2];
    void index() const {
        std::lock_guard<std::mutex> g(mu);
        if (indexed) return;
        for (const Key &k : set) {
            by_side[0][{k.t, k.r}].push_back(k.h);
            by_side[1][{k.h, k.r}].push_back(k.t);
        }
        indexed = true;
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
    for (int64_t i = 0; i < n; ++i) k->set.insert(Key{h[i], t[i], r[i]});
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
    const auto &m = k->by_side[side];
    off[0] = 0;
    for (int64_t q = 0; q < n; ++q) {
        const auto it = m.find({anchor[q], rel[q]});
        int64_t c = 0;
        if (it != m.end()) {
            for (int64_t e : it->second) {
                if (list) list[off[q] + c] = e;
                ++c;
            }
        }
        if (list) std::sort(list + off[q], list + off[q] + c);   // ascending: pt_rank_types bisects it
        off[q + 1] = off[q] + c;
    }
    return PT_OK;
}
