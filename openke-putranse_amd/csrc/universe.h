// Parallel-universe training sets (UniverseConstructor.h / UniverseSetting.h of the reference).
#pragma once
#include <cstdint>
#include <vector>

#include "graph.h"
#include "rng.h"

namespace pt {

struct Universe {
    Graph g;                         // local ids, helpers as loadUniverseHelpers builds them
    std::vector<int64_t> ent_remap;  // local -> global (getEntityRemapping)
    std::vector<int64_t> rel_remap;  // local -> global (getRelationRemapping)
    std::vector<uint64_t> seeds;     // per-thread LCG states drawn by randReset before construction
    int64_t focus = -1;
};

// getParallelUniverse(tc, balance) continuing the glibc stream `rng` (UniverseConstructor.h:327-397)
void build_universe(const Graph &global, GlibcRand &rng, int64_t triple_constraint, float balance, Universe &u);

}  // namespace pt

struct pt_universe {
    pt::Universe u;
};
