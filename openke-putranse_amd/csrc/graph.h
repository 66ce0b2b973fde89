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

// One training triple as the sampler needs it (ids as int32: every benchmark id fits). hr_lo/hr_hi
// bound the triple's (h,r) run in the cmp_head list and tr_lo/tr_hi its (t,r) run in the cmp_tail
// list: exactly the [ll, rr] the reference finds with two binary searches per filtered corruption
// (Corrupt.h:27-42, :75-90), precomputed once so a corruption costs one dependent load, not ~2 log n.
struct TripleRec {
    int32_t h, r, t, hr_lo, hr_hi, tr_lo, tr_hi, pad;
};

// Device mirror consumed by the kernels.
struct DeviceGraph {
    int64_t ent_total = 0, rel_total = 0, train_total = 0;
    const TripleRec *rec = nullptr;     // cmp_head order (trainList == trainHead after the reader's sort)
    const int32_t *head_t = nullptr;    // trainHead[k].t: values corrupt_head searches
    const int32_t *tail_h = nullptr;    // trainTail[k].h: values corrupt_tail searches
    const float *bern_prob = nullptr;   // per relation: 1000*right_mean/(right_mean+left_mean) (Base.cpp:219-221)
    const int32_t *rel_r = nullptr;     // trainRel[k].r (cmp_rel order): values corrupt_rel searches
    const int2 *ht_run = nullptr;       // per triple (head order): its (h,t) run [ll, rr] in the cmp_rel list
};

struct Graph {
    int64_t ent_total = 0, rel_total = 0, train_total = 0;
    std::vector<Triple> list, head, tail, rel, rel2;   // cmp_head / cmp_head / cmp_tail / cmp_rel / cmp_rel2
    std::vector<int64_t> lef_head, rig_head, lef_tail, rig_tail, lef_rel, rig_rel, lef_rel2, rig_rel2;
    std::vector<int64_t> freq_ent, freq_rel;
    std::vector<float> left_mean, right_mean;

    // device copy (lazily uploaded to the current device)
    bool ht_full = false;                 // some (h,t) pair holds every relation: corrupt_rel would divide by 0
    int device = -1;
    void *dev_block = nullptr;
    DeviceGraph dev;

    ~Graph();
    void build_helpers();                 // loadHelpers / loadUniverseHelpers (Reader.h:58-167)
    int upload();                         // PT_OK or error; idempotent
    // the device image of the graph as host bytes (layout of DeviceGraph, 256-byte aligned parts; sets
    // ht_full) and the DeviceGraph of that image placed at device address `base` (upload() = image + one
    // allocation + bind; a universe set places many images in one allocation)
    std::vector<char> device_image();
    DeviceGraph bind_image(char *base) const;
};

int load_graph(const std::string &dir, Graph &g);   // importTrainFiles (Reader.h:169-234)
int64_t count_lines(const std::string &path, bool *ok);

// Record-file format. Default (false): the record count is the line count and every line is a record,
// the reference's contract (Reader.h:176-196). true: the first line holds the record count (the
// upstream OpenKE / benchmark count-header format) and the records follow it.
void set_count_header(bool on);
bool count_header();
// Number of records in a *2id.txt file under the current format (0 and *ok=false when unreadable; a
// malformed header also sets *ok=false and fills *err).
int64_t record_count(const std::string &path, bool *ok, std::string *err = nullptr);
// n "a b c" triples (file order h t r) after the header line when the count-header format is on.
bool read_triples(const std::string &path, int64_t n, std::vector<Triple> &out);

bool cmp_head(const Triple &a, const Triple &b);
bool cmp_tail(const Triple &a, const Triple &b);
bool cmp_rel(const Triple &a, const Triple &b);
bool cmp_rel2(const Triple &a, const Triple &b);

}  // namespace pt

struct pt_graph {
    pt::Graph g;
};
