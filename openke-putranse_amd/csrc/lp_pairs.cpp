// (key, universe) pairs of a global energy estimation (host only): for every evaluation key (side, anchor
// entity, relation) the universes holding both the anchor and the relation, with the universe-local ids - the
// universes Parallel_Universe_Config.eval_universes scores for that key (Parallel_Universe_Config.py:470-476),
// as the pt_lp_pair rows pt_lp_min_scores takes. An inverted index of the universes' entities by global id
// (counting sort, universe order kept) joined with the keys; the relation tested in the universe's sorted
// relation list: a dense (universe, global relation) -> local table when it is small (C4: 1,024 x 121 entries), else
// a binary search in the universe's sorted relations. The keys are joined on up to 16 host threads, each over a
// contiguous key range, and the ranges' rows concatenated in key order: the same rows in the same order as one
// thread (tests/test_native_cpu.py).
#include <algorithm>
#include <cstring>
#include <thread>
#include <utility>
#include <vector>

#include "putranse.h"

namespace {

bool csr_ok(int64_t n, const int64_t *off, const int64_t *ids) {
    if (n && (!off || off[0] != 0)) return false;
    for (int64_t u = 0; u < n; ++u)
        if (off[u + 1] < off[u]) return false;
    const int64_t m = n ? off[n] : 0;
    if (m && !ids) return false;
    for (int64_t i = 0; i < m; ++i)
        if (ids[i] < 0 || ids[i] >= (int64_t(1) << 31)) return false;
    return true;
}

}  // namespace

extern "C" int pt_lp_pairs(int64_t n, const int64_t *ent_off, const int64_t *ent_ids, const int64_t *rel_off,
                           const int64_t *rel_ids, int64_t n_keys, const int64_t *key_anchor, const int64_t *key_rel,
                           const int64_t *key_side, pt_lp_pair *out, int64_t cap, int64_t *n_out) {
    if (!n_out || n < 0 || n >= (int64_t(1) << 31) || n_keys < 0 || n_keys >= (int64_t(1) << 31)) return PT_EINVAL;
    if (!csr_ok(n, ent_off, ent_ids) || !csr_ok(n, rel_off, rel_ids)) return PT_EINVAL;
    if (n_keys && (!key_anchor || !key_rel || !key_side)) return PT_EINVAL;
    const int64_t m = n ? ent_off[n] : 0;
    int64_t bound = 0;
    for (int64_t i = 0; i < m; ++i) bound = std::max(bound, ent_ids[i] + 1);
    std::vector<int64_t> start(bound + 1, 0);
    for (int64_t i = 0; i < m; ++i) ++start[ent_ids[i] + 1];
    for (int64_t g = 0; g < bound; ++g) start[g + 1] += start[g];
    if (!out) {   // an upper bound: the (key, universe holding the anchor) pairs
        int64_t ub = 0;
        for (int64_t k = 0; k < n_keys; ++k) {
            const int64_t a = key_anchor[k];
            if (a >= 0 && a < bound) ub += start[a + 1] - start[a];
        }
        *n_out = ub;
        return PT_OK;
    }
    std::vector<int64_t> fill(start.begin(), start.end() - 1);
    std::vector<int32_t> occ_u(m), occ_l(m);
    for (int64_t u = 0; u < n; ++u)
        for (int64_t i = ent_off[u]; i < ent_off[u + 1]; ++i) {
            const int64_t j = fill[ent_ids[i]]++;
            occ_u[j] = static_cast<int32_t>(u);
            occ_l[j] = static_cast<int32_t>(i - ent_off[u]);
        }
    // each universe's relations: a dense global -> local table, or (global, local) pairs sorted by global id
    const int64_t nr = n ? rel_off[n] : 0;
    int64_t rbound = 0;
    for (int64_t i = 0; i < nr; ++i) rbound = std::max(rbound, rel_ids[i] + 1);
    const bool dense = n * rbound <= (int64_t(1) << 24);
    std::vector<int32_t> rtab(dense ? (size_t)(n * rbound) : 0, -1);
    std::vector<std::pair<int64_t, int32_t>> rel(dense ? 0 : nr);
    for (int64_t u = 0; u < n; ++u) {
        for (int64_t i = rel_off[u]; i < rel_off[u + 1]; ++i) {
            const int32_t loc = static_cast<int32_t>(i - rel_off[u]);
            if (dense) {
                int32_t &t = rtab[(size_t)(u * rbound + rel_ids[i])];
                if (t < 0) t = loc;   // (a repeated relation id: its first local id, as lower_bound finds)
            } else {
                rel[i] = {rel_ids[i], loc};
            }
        }
        if (!dense) std::sort(rel.begin() + rel_off[u], rel.begin() + rel_off[u + 1]);
    }
    auto local_rel = [&](int32_t u, int64_t r) -> int32_t {
        if (dense) return r >= 0 && r < rbound ? rtab[(size_t)(u * rbound + r)] : -1;
        const auto lo = rel.begin() + rel_off[u], hi = rel.begin() + rel_off[u + 1];
        const auto it = std::lower_bound(lo, hi, std::make_pair(r, INT32_MIN));
        return it == hi || it->first != r ? -1 : it->second;
    };
    auto join = [&](int64_t k0, int64_t k1, std::vector<pt_lp_pair> &rows) {
        for (int64_t k = k0; k < k1; ++k) {
            const int64_t a = key_anchor[k], r = key_rel[k];
            if (a < 0 || a >= bound) continue;
            for (int64_t j = start[a]; j < start[a + 1]; ++j) {
                const int32_t u = occ_u[j];
                const int32_t lr = local_rel(u, r);
                if (lr < 0) continue;
                rows.push_back(pt_lp_pair{static_cast<int32_t>(k), u, occ_l[j], lr, static_cast<int32_t>(key_side[k])});
            }
        }
    };
    const int64_t nt = n_keys < 4096 ? 1 : std::min<int64_t>(16, std::max(1u, std::thread::hardware_concurrency()));
    std::vector<std::vector<pt_lp_pair>> part((size_t)nt);
    if (nt == 1) {
        join(0, n_keys, part[0]);
    } else {
        std::vector<std::thread> pool;
        for (int64_t t = 0; t < nt; ++t)
            pool.emplace_back([&, t] { join(n_keys * t / nt, n_keys * (t + 1) / nt, part[(size_t)t]); });
        for (auto &th : pool) th.join();
    }
    int64_t w = 0;
    for (const auto &rows : part) {
        if (w + (int64_t)rows.size() > cap) return PT_EINVAL;
        if (!rows.empty()) std::memcpy(out + w, rows.data(), rows.size() * sizeof(pt_lp_pair));
        w += (int64_t)rows.size();
    }
    *n_out = w;
    return PT_OK;
}
