// Training graph: deduplicated triples + the reference's helper indices, host and device copies.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "common.h"

namespace pt {

struct Triple {
    int64_t h, r, t;
};

// Device mirror consumed by the kernels (ids as int32: every benchmark id fits, halves the bytes).
struct DeviceGraph {
    int64_t ent_total = 0, rel_total = 0, train_total = 0;
    const int32_t *list_h = nullptr, *list_r = nullptr, *list_t = nullptr;   // cmp_head order (= trainHead)
    const int32_t *tail_h = nullptr, *tail_r = nullptr;                      // cmp_tail order (trainTail)
    const int32_t *lef_head = nullptr, *rig_head = nullptr, *lef_tail = nullptr, *rig_tail = nullptr;
    const float *bern_prob = nullptr;   // per relation: 1000*right_mean/(right_mean+left_mean) (Base.cpp:219-221)
};

struct Graph {
    int64_t ent_total = 0, rel_total = 0, train_total = 0;
    std::vector<Triple> list, head, tail, rel, rel2;   // cmp_head / cmp_head / cmp_tail / cmp_rel / cmp_rel2
    std::vector<int64_t> lef_head, rig_head, lef_tail, rig_tail, lef_rel, rig_rel, lef_rel2, rig_rel2;
    std::vector<int64_t> freq_ent, freq_rel;
    std::vector<float> left_mean, right_mean;

    // device copy (lazily uploaded to the current device)
    int device = -1;
    void *dev_block = nullptr;
    DeviceGraph dev;

    ~Graph();
    void build_helpers();                 // loadHelpers / loadUniverseHelpers (Reader.h:58-167)
    int upload();                         // PT_OK or error; idempotent
};

int load_graph(const std::string &dir, Graph &g);   // importTrainFiles (Reader.h:169-234)
int64_t count_lines(const std::string &path, bool *ok);

bool cmp_head(const Triple &a, const Triple &b);
bool cmp_tail(const Triple &a, const Triple &b);
bool cmp_rel(const Triple &a, const Triple &b);
bool cmp_rel2(const Triple &a, const Triple &b);

}  // namespace pt

struct pt_graph {
    pt::Graph g;
};
