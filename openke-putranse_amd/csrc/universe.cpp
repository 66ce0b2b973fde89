// Universe construction: relation focus -> entity subsample -> bidirectional random walk ->
// local re-enumeration -> helpers. Output is identical to getParallelUniverse
// (UniverseConstructor.h:327-397) for the same glibc stream; the data structures are chosen for
// speed (hash set for the duplicate test the reference does by linear scan, Fenwick-tree selection
// for the random subset), which changes no draw and no result.
#include "universe.h"

#include <algorithm>
#include <set>
#include <unordered_set>

namespace pt {

namespace {

// k-th smallest alive element with deletion, O(log n) (get_entity_subset, :55-67, draws
// std::advance(begin, rand() % size) over a shrinking ordered set)
struct AliveSelect {
    std::vector<int64_t> vals;
    std::vector<int32_t> bit;
    int64_t alive = 0;
    int top = 1;
    explicit AliveSelect(std::vector<int64_t> v) : vals(std::move(v)) {
        const int64_t n = (int64_t)vals.size();
        bit.assign((size_t)n + 1, 0);
        for (int64_t i = 1; i <= n; ++i) {
            bit[i] += 1;
            int64_t j = i + (i & -i);
            if (j <= n) bit[j] += bit[i];
        }
        alive = n;
        while ((top << 1) <= n) top <<= 1;
    }
    int64_t take(int64_t k) {   // 0-based rank among alive; removes it
        int64_t pos = 0, rem = k + 1;
        const int64_t n = (int64_t)vals.size();
        for (int step = top; step; step >>= 1) {
            if (pos + step <= n && bit[pos + step] < rem) {
                pos += step;
                rem -= bit[pos];
            }
        }
        int64_t idx = pos;   // 0-based index of the element
        for (int64_t i = idx + 1; i <= n; i += i & -i) bit[i] -= 1;
        --alive;
        return vals[(size_t)idx];
    }
};

struct TripleHash {
    size_t operator()(const Triple &x) const {
        uint64_t k = (uint64_t)x.h * 0x9E3779B97F4A7C15ULL ^ ((uint64_t)x.r << 40) ^ (uint64_t)x.t * 0xC2B2AE3D27D4EB4FULL;
        return (size_t)(k ^ (k >> 29));
    }
};
struct TripleEq {
    bool operator()(const Triple &a, const Triple &b) const { return a.h == b.h && a.r == b.r && a.t == b.t; }
};

}  // namespace

void build_universe(const Graph &G, GlibcRand &rng, int64_t tc, float balance, Universe &u) {
    int64_t target = tc;
    std::vector<Triple> walk;
    walk.reserve((size_t)std::max<int64_t>(tc, 0));
    const int64_t focus = rng.range(0, G.rel_total);                      // :336-342
    u.focus = focus;
    const int64_t threshold = (int64_t)(balance * (float)tc);              // :343-344 (float product)

    // entities of the focus relation (gatherRelationEntities, :69-80), ascending
    std::vector<int64_t> ents;
    for (int64_t k = G.lef_rel2[focus]; k < G.rig_rel2[focus] + 1; ++k) {
        ents.push_back(G.rel2[k].h);
        ents.push_back(G.rel2[k].t);
    }
    std::sort(ents.begin(), ents.end());
    ents.erase(std::unique(ents.begin(), ents.end()), ents.end());
    std::set<int64_t> S;
    if ((uint64_t)ents.size() > (uint64_t)threshold) {                    // :352-354
        AliveSelect sel(ents);
        while ((int64_t)S.size() < threshold) {
            int64_t k = (int64_t)((uint64_t)(int64_t)rng.next() % (uint64_t)sel.alive);
            S.insert(sel.take(k));
        }
    } else {
        S.insert(ents.begin(), ents.end());
    }

    // BidirectionalRandomWalk (:92-191)
    std::unordered_set<Triple, TripleHash, TripleEq> seen;
    seen.reserve((size_t)std::max<int64_t>(2 * tc, 16));
    std::set<int64_t> nsp, uent, urel;
    int64_t last_dup = -1, tol = 5, not_inc = 20, last_size = 0;
    while ((int64_t)walk.size() < target) {
        auto it = S.begin();
        while (it != S.end() && (int64_t)walk.size() < target) {
            const int64_t cur = *it;
            Triple x{0, 0, 0};
            int64_t start = -1;
            int from_head;
            if (rng.next() % 1000 < 500)
                from_head = G.rig_head[cur] != -1 ? 1 : (G.rig_tail[cur] != -1 ? 0 : -1);
            else
                from_head = G.rig_tail[cur] != -1 ? 0 : (G.rig_head[cur] != -1 ? 1 : -1);
            if (from_head == 1) {          // gatherTripleFromHead (:39-45)
                x = G.head[rng.range(G.lef_head[cur], G.rig_head[cur] + 1)];
                start = x.t;
            } else if (from_head == 0) {   // gatherTripleFromTail (:47-53)
                x = G.tail[rng.range(G.lef_tail[cur], G.rig_tail[cur] + 1)];
                start = x.h;
            }
            if (seen.count(x)) {           // duplicate: per-entity retry tolerance (:141-153)
                if (last_dup == cur) tol--; else last_dup = cur;
                if (tol == 0) {
                    tol = 5;
                    ++it;
                }
                continue;
            }
            seen.insert(x);
            walk.push_back(x);
            nsp.insert(start);
            uent.insert(x.t);
            uent.insert(x.h);
            urel.insert(x.r);
            it = S.erase(it);
        }
        S.swap(nsp);   // leftovers of this round stay in nsp for the next (as the reference's swap)
        const int64_t got = (int64_t)walk.size();
        if (got == last_size) not_inc--; else { last_size = got; not_inc = 20; }
        if (not_inc == 0) {
            target = got;
            break;
        }
    }

    // enumerateTrainUniverseTriples (:193-233): local ids by first appearance h, t, r
    Graph &L = u.g;
    L.ent_total = (int64_t)uent.size();
    L.rel_total = (int64_t)urel.size();
    L.train_total = (int64_t)walk.size();
    std::vector<int64_t> emap((size_t)G.ent_total, -1), rmap((size_t)G.rel_total, -1);
    u.ent_remap.assign((size_t)L.ent_total, -1);
    u.rel_remap.assign((size_t)L.rel_total, -1);
    int64_t ne = 0, nr = 0;
    L.list.resize(walk.size());
    for (size_t i = 0; i < walk.size(); ++i) {
        const Triple &w = walk[i];
        if (emap[w.h] == -1) { emap[w.h] = ne; u.ent_remap[ne++] = w.h; }
        if (emap[w.t] == -1) { emap[w.t] = ne; u.ent_remap[ne++] = w.t; }
        if (rmap[w.r] == -1) { rmap[w.r] = nr; u.rel_remap[nr++] = w.r; }
        L.list[i] = Triple{emap[w.h], rmap[w.r], emap[w.t]};
    }
    L.build_helpers();   // loadUniverseHelpers (:235-325)
}

}  // namespace pt
