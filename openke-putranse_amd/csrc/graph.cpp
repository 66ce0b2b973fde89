// Training-graph ingest and helper indices (replaces Reader.h:58-234 importTrainFiles/loadHelpers).
#include "graph.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>

namespace pt {

bool cmp_head(const Triple &a, const Triple &b) {   // Triple.h:7-9
    return a.h != b.h ? a.h < b.h : (a.r != b.r ? a.r < b.r : a.t < b.t);
}
bool cmp_tail(const Triple &a, const Triple &b) {   // Triple.h:11-13
    return a.t != b.t ? a.t < b.t : (a.r != b.r ? a.r < b.r : a.h < b.h);
}
bool cmp_rel(const Triple &a, const Triple &b) {    // Triple.h:15-17
    return a.h != b.h ? a.h < b.h : (a.t != b.t ? a.t < b.t : a.r < b.r);
}
bool cmp_rel2(const Triple &a, const Triple &b) {   // Triple.h:19-21
    return a.r != b.r ? a.r < b.r : (a.h != b.h ? a.h < b.h : a.t < b.t);
}

Graph::~Graph() {
    if (dev_block) {
        int cur = 0;
        if (hipGetDevice(&cur) == hipSuccess && cur != device) {
            (void)hipSetDevice(device);
            (void)hipFree(dev_block);
            (void)hipSetDevice(cur);
        } else {
            (void)hipFree(dev_block);
        }
    }
}

// The line count is the record count: the reference never reads the count header (Reader.h:176-196,
// Utilities.h:47-57), so we keep that contract for drop-in parity on headerless benchmark folders.
int64_t count_lines(const std::string &path, bool *ok) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) {
        *ok = false;
        return 0;
    }
    int64_t n = 0;
    char buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0)
        for (size_t i = 0; i < k; ++i) n += buf[i] == '\n';
    fclose(f);
    *ok = true;
    return n;
}

static std::atomic<bool> g_count_header{false};
void set_count_header(bool on) { g_count_header.store(on); }
bool count_header() { return g_count_header.load(); }

// Header line of a count-header file: exactly one non-negative integer (upstream OpenKE reads it with
// fscanf("%ld"), the call this fork commented out at Reader.h:178/185/191).
int64_t record_count(const std::string &path, bool *ok, std::string *err) {
    if (!count_header()) return count_lines(path, ok);
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) {
        *ok = false;
        return 0;
    }
    char line[256] = {0};
    const bool got = fgets(line, sizeof line, f) != nullptr;
    fclose(f);
    char *end = nullptr;
    const long long v = got ? strtoll(line, &end, 10) : -1;
    bool good = got && end != line && v >= 0;
    for (const char *p = end; good && p && *p; ++p)
        if (!(*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) good = false;
    if (!good) {
        *ok = false;
        if (err) *err = "count-header format: first line of " + path + " is not a record count";
        return 0;
    }
    *ok = true;
    return (int64_t)v;
}

bool read_triples(const std::string &path, int64_t n, std::vector<Triple> &out) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    out.resize((size_t)n);
    // hand-rolled integer scanner (fscanf per field dominates ingest time on 10^6-line files)
    std::vector<char> data;
    {
        fseek(f, 0, SEEK_END);
        long sz = ftell(f);
        fseek(f, 0, SEEK_SET);
        data.resize((size_t)sz + 1);
        size_t got = fread(data.data(), 1, (size_t)sz, f);
        data[got] = 0;
    }
    fclose(f);
    const char *p = data.data();
    if (count_header()) {   // skip the count line
        while (*p && *p != '\n') ++p;
        if (*p) ++p;
    }
    auto next_int = [&](int64_t &v) -> bool {
        while (*p && !(*p == '-' || (*p >= '0' && *p <= '9'))) ++p;
        if (!*p) return false;
        bool neg = *p == '-';
        if (neg) ++p;
        int64_t x = 0;
        while (*p >= '0' && *p <= '9') x = x * 10 + (*p++ - '0');
        v = neg ? -x : x;
        return true;
    };
    for (int64_t i = 0; i < n; ++i) {
        Triple &tr = out[(size_t)i];
        if (!next_int(tr.h) || !next_int(tr.t) || !next_int(tr.r)) {   // file order: h t r
            out.resize((size_t)i);
            return true;
        }
    }
    return true;
}

void Graph::build_helpers() {
    const int64_t n = train_total, E = ent_total, R = rel_total;
    std::sort(list.begin(), list.end(), cmp_head);
    head = tail = rel = rel2 = list;
    freq_ent.assign((size_t)E, 0);
    freq_rel.assign((size_t)R, 0);
    for (const Triple &x : list) {
        freq_ent[(size_t)x.h]++;
        freq_ent[(size_t)x.t]++;
        freq_rel[(size_t)x.r]++;
    }
    // head == list already (cmp_head)
    std::sort(tail.begin(), tail.end(), cmp_tail);
    std::sort(rel.begin(), rel.end(), cmp_rel);
    std::sort(rel2.begin(), rel2.end(), cmp_rel2);
    lef_head.assign((size_t)E, 0); rig_head.assign((size_t)E, -1);
    lef_tail.assign((size_t)E, 0); rig_tail.assign((size_t)E, -1);
    lef_rel.assign((size_t)E, 0);  rig_rel.assign((size_t)E, -1);
    lef_rel2.assign((size_t)R, 0); rig_rel2.assign((size_t)R, -1);
    for (int64_t i = 1; i < n; ++i) {
        if (tail[i].t != tail[i - 1].t) { rig_tail[tail[i - 1].t] = i - 1; lef_tail[tail[i].t] = i; }
        if (head[i].h != head[i - 1].h) { rig_head[head[i - 1].h] = i - 1; lef_head[head[i].h] = i; }
        if (rel[i].h != rel[i - 1].h) { rig_rel[rel[i - 1].h] = i - 1; lef_rel[rel[i].h] = i; }
        if (rel2[i].r != rel2[i - 1].r) { rig_rel2[rel2[i - 1].r] = i - 1; lef_rel2[rel2[i].r] = i; }
    }
    if (n > 0) {
        lef_head[head[0].h] = 0; rig_head[head[n - 1].h] = n - 1;
        lef_tail[tail[0].t] = 0; rig_tail[tail[n - 1].t] = n - 1;
        lef_rel[rel[0].h] = 0;   rig_rel[rel[n - 1].h] = n - 1;
        lef_rel2[rel2[0].r] = 0; rig_rel2[rel2[n - 1].r] = n - 1;
    }
    // relation-wise mean #tails per head (left) and #heads per tail (right), Reader.h:148-166
    left_mean.assign((size_t)R, 0.f);
    right_mean.assign((size_t)R, 0.f);
    for (int64_t i = 0; i < E; ++i) {
        for (int64_t j = lef_head[i] + 1; j <= rig_head[i]; ++j)
            if (head[j].r != head[j - 1].r) left_mean[head[j].r] += 1.0f;
        if (lef_head[i] <= rig_head[i]) left_mean[head[lef_head[i]].r] += 1.0f;
        for (int64_t j = lef_tail[i] + 1; j <= rig_tail[i]; ++j)
            if (tail[j].r != tail[j - 1].r) right_mean[tail[j].r] += 1.0f;
        if (lef_tail[i] <= rig_tail[i]) right_mean[tail[lef_tail[i]].r] += 1.0f;
    }
    for (int64_t i = 0; i < R; ++i) {
        left_mean[i] = (float)freq_rel[i] / left_mean[i];
        right_mean[i] = (float)freq_rel[i] / right_mean[i];
    }
}

int load_graph(const std::string &dir, Graph &g) {
    bool ok = true;
    std::string err;
    g.rel_total = record_count(dir + "relation2id.txt", &ok, &err);
    PT_CHECK(ok, PT_EIO, err.empty() ? "cannot open " + dir + "relation2id.txt" : err);
    g.ent_total = record_count(dir + "entity2id.txt", &ok, &err);
    PT_CHECK(ok, PT_EIO, err.empty() ? "cannot open " + dir + "entity2id.txt" : err);
    int64_t n = record_count(dir + "train2id.txt", &ok, &err);
    PT_CHECK(ok, PT_EIO, err.empty() ? "cannot open " + dir + "train2id.txt" : err);
    PT_CHECK(read_triples(dir + "train2id.txt", n, g.list), PT_EIO, "cannot read " + dir + "train2id.txt");
    PT_CHECK(!count_header() || (int64_t)g.list.size() == n, PT_EIO,
             "count-header format: " + dir + "train2id.txt holds fewer triples than its header says");
    const char *hint = count_header() ? "" : " (count-header file? see pt_set_count_header)";
    for (const Triple &x : g.list)
        PT_CHECK(x.h >= 0 && x.t >= 0 && x.r >= 0 && x.h < g.ent_total && x.t < g.ent_total && x.r < g.rel_total,
                 PT_EIO, "triple id out of range in " + dir + "train2id.txt" + hint);
    std::sort(g.list.begin(), g.list.end(), cmp_head);
    g.list.erase(std::unique(g.list.begin(), g.list.end(),
                             [](const Triple &a, const Triple &b) { return a.h == b.h && a.r == b.r && a.t == b.t; }),
                 g.list.end());
    g.train_total = (int64_t)g.list.size();
    PT_CHECK(g.train_total > 0, PT_EIO, "empty training set in " + dir);
    g.build_helpers();
    return PT_OK;
}

namespace {
struct ImageLayout {
    size_t rec, ht, th, bp, rr, hr, total;
    ImageLayout(int64_t n, int64_t R) {
        auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
        rec = 0;
        ht = rec + al(sizeof(TripleRec) * n);
        th = ht + al(4 * n);
        bp = th + al(4 * n);
        rr = bp + al(4 * (R ? R : 1));
        hr = rr + al(4 * n);
        total = hr + al(8 * n);
    }
};
}  // namespace

std::vector<char> Graph::device_image() {
    const int64_t n = train_total, R = rel_total;
    const ImageLayout L(n, R);
    std::vector<TripleRec> rec((size_t)n);
    // (h,r) runs of the cmp_head list
    for (int64_t i = 0; i < n;) {
        int64_t j = i;
        while (j + 1 < n && list[j + 1].h == list[i].h && list[j + 1].r == list[i].r) ++j;
        for (int64_t k = i; k <= j; ++k) {
            rec[k] = TripleRec{(int32_t)list[k].h, (int32_t)list[k].r, (int32_t)list[k].t, (int32_t)i, (int32_t)j,
                               0, 0, 0};
        }
        i = j + 1;
    }
    // (t,r) runs of the cmp_tail list, mapped back to head order
    std::vector<int64_t> order((size_t)n);
    for (int64_t i = 0; i < n; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return cmp_tail(list[a], list[b]); });
    for (int64_t i = 0; i < n;) {
        int64_t j = i;
        while (j + 1 < n && tail[j + 1].t == tail[i].t && tail[j + 1].r == tail[i].r) ++j;
        for (int64_t k = i; k <= j; ++k) {
            rec[order[k]].tr_lo = (int32_t)i;
            rec[order[k]].tr_hi = (int32_t)j;
        }
        i = j + 1;
    }
    std::vector<char> host(L.total, 0);
    memcpy(host.data() + L.rec, rec.data(), sizeof(TripleRec) * n);
    int32_t *ht = (int32_t *)(host.data() + L.ht), *th = (int32_t *)(host.data() + L.th);
    for (int64_t i = 0; i < n; ++i) {
        ht[i] = (int32_t)head[i].t;
        th[i] = (int32_t)tail[i].h;
    }
    // corrupt_rel (Corrupt.h:108-189): the relations of the cmp_rel list and, per triple in head order,
    // the (h,t) run [ll, rr] its two binary searches find
    int32_t *rr_col = (int32_t *)(host.data() + L.rr), *hr_run = (int32_t *)(host.data() + L.hr);
    std::vector<int64_t> rorder((size_t)n);
    for (int64_t i = 0; i < n; ++i) rorder[i] = i;
    std::sort(rorder.begin(), rorder.end(), [&](int64_t a, int64_t b) { return cmp_rel(list[a], list[b]); });
    ht_full = false;
    for (int64_t i = 0; i < n;) {
        int64_t j = i;
        while (j + 1 < n && rel[j + 1].h == rel[i].h && rel[j + 1].t == rel[i].t) ++j;
        for (int64_t k = i; k <= j; ++k) {
            rr_col[k] = (int32_t)rel[k].r;
            hr_run[2 * rorder[k]] = (int32_t)i;
            hr_run[2 * rorder[k] + 1] = (int32_t)j;
        }
        if (j - i + 1 >= R) ht_full = true;
        i = j + 1;
    }
    float *bp = (float *)(host.data() + L.bp);
    for (int64_t r = 0; r < R; ++r) bp[r] = 1000 * right_mean[r] / (right_mean[r] + left_mean[r]);
    return host;
}

DeviceGraph Graph::bind_image(char *b) const {
    const ImageLayout L(train_total, rel_total);
    DeviceGraph d;
    d.ent_total = ent_total;
    d.rel_total = rel_total;
    d.train_total = train_total;
    d.rec = (const TripleRec *)(b + L.rec);
    d.head_t = (const int32_t *)(b + L.ht);
    d.tail_h = (const int32_t *)(b + L.th);
    d.bern_prob = (const float *)(b + L.bp);
    d.rel_r = (const int32_t *)(b + L.rr);
    d.ht_run = (const int2 *)(b + L.hr);
    return d;
}

int Graph::upload() {
    int cur = 0;
    PT_HIP(hipGetDevice(&cur));
    if (dev_block && device == cur) return PT_OK;
    PT_CHECK(!dev_block, PT_ESTATE, "graph already uploaded to another device");
    const std::vector<char> host = device_image();
    PT_HIP(hipMalloc(&dev_block, host.size()));
    PT_HIP(hipMemcpy(dev_block, host.data(), host.size(), hipMemcpyHostToDevice));
    dev = bind_image((char *)dev_block);
    device = cur;
    return PT_OK;
}

}  // namespace pt
