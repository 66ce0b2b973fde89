// (key, universe) pairs of a global energy estimation (host only): for every evaluation key (side, anchor
// entity, relation) the universes holding both the anchor and the relation, with the universe-local ids - the
// universes Parallel_Universe_Config.eval_universes scores for that key (Parallel_Universe_Config.py:470-476),
// as the pt_lp_pair rows pt_lp_min_scores takes. An inverted index of the universes' entities by global id
// (counting sort, universe order kept) joined with the keys; the relation tested in the universe's sorted
// relation list.
#include <algorithm>
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
    // each universe's relations as (global, local), sorted by global id
    std::vector<std::pair<int64_t, int32_t>> rel(n ? rel_off[n] : 0);
    for (int64_t u = 0; u < n; ++u) {
        for (int64_t i = rel_off[u]; i < rel_off[u + 1]; ++i)
            rel[i] = {rel_ids[i], static_cast<int32_t>(i - rel_off[u])};
        std::sort(rel.begin() + rel_off[u], rel.begin() + rel_off[u + 1]);
    }
    int64_t w = 0;
    for (int64_t k = 0; k < n_keys; ++k) {
        const int64_t a = key_anchor[k], r = key_rel[k];
        if (a < 0 || a >= bound) continue;
        for (int64_t j = start[a]; j < start[a + 1]; ++j) {
            const int32_t u = occ_u[j];
            const auto lo = rel.begin() + rel_off[u], hi = rel.begin() + rel_off[u + 1];
            const auto it = std::lower_bound(lo, hi, std::make_pair(r, INT32_MIN));
            if (it == hi || it->first != r) continue;
            if (w >= cap) return PT_EINVAL;
            out[w++] = pt_lp_pair{static_cast<int32_t>(k), u, occ_l[j], it->second, static_cast<int32_t>(key_side[k])};
        }
    }
    *n_out = w;
    return PT_OK;
}
