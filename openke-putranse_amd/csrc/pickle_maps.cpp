// Checkpoint encoding of the universe id maps (host only): the item regions of the pickle streams that
// openke/config/_map_pickle.py wraps into entity_id_mappings / relation_id_mappings / entity_universes /
// relation_universes (the reference's dictionaries, Parallel_Universe_Config.py:90-95, filled by
// process_universe_mappings :179-207 and written by save_parameters :890-899). One pass over the remap arrays
// instead of building the Python dictionaries and pickling them.
#include <cstring>
#include <vector>

#include "putranse.h"

namespace {

// BININT: 'J' + little-endian int32
inline uint8_t *put_int(uint8_t *p, int64_t v) {
    const int32_t x = static_cast<int32_t>(v);
    *p++ = 'J';
    std::memcpy(p, &x, 4);
    return p + 4;
}

bool ids_ok(int64_t n, const int64_t *uids, const int64_t *off, const int64_t *ids) {
    if (n < 0 || (n && (!uids || !off))) return false;
    if (n && off[0] != 0) return false;
    for (int64_t u = 0; u < n; ++u) {
        if (off[u + 1] < off[u] || uids[u] < 0 || uids[u] >= (int64_t(1) << 31)) return false;
        if (u && uids[u] <= uids[u - 1]) return false;
    }
    const int64_t m = n ? off[n] : 0;
    if (m && !ids) return false;
    for (int64_t i = 0; i < m; ++i)
        if (ids[i] < 0 || ids[i] >= (int64_t(1) << 31)) return false;
    return true;
}

}  // namespace

extern "C" int pt_pickle_id_maps(int64_t n, const int64_t *uids, const int64_t *off, const int64_t *ids, uint8_t *out,
                                 int64_t cap, int64_t *n_out) {
    if (!n_out || !ids_ok(n, uids, off, ids)) return PT_EINVAL;
    // per universe: J uid, BINGET 0, BINGET 1, TUPLE1, REDUCE [, MARK, (J id, J local) * n, SETITEMS]
    int64_t need = 0;
    for (int64_t u = 0; u < n; ++u) {
        const int64_t k = off[u + 1] - off[u];
        need += 11 + (k ? 2 + 10 * k : 0);
    }
    *n_out = need;
    if (!out) return PT_OK;
    if (cap < need) return PT_EINVAL;
    uint8_t *p = out;
    for (int64_t u = 0; u < n; ++u) {
        p = put_int(p, uids[u]);
        const uint8_t head[4] = {'h', 0, 'h', 1};
        std::memcpy(p, head, 4);
        p += 4;
        *p++ = 0x85;   // TUPLE1
        *p++ = 'R';    // REDUCE: defaultdict(int)
        const int64_t k = off[u + 1] - off[u];
        if (!k) continue;
        *p++ = '(';
        for (int64_t i = 0; i < k; ++i) {
            p = put_int(p, ids[off[u] + i]);
            p = put_int(p, i);
        }
        *p++ = 'u';   // SETITEMS
    }
    return PT_OK;
}

extern "C" int pt_pickle_universe_sets(int64_t n, const int64_t *uids, const int64_t *off, const int64_t *ids,
                                       uint8_t *out, int64_t cap, int64_t *n_out) {
    if (!n_out || !ids_ok(n, uids, off, ids)) return PT_EINVAL;
    const int64_t m = n ? off[n] : 0;
    int64_t bound = 0;
    for (int64_t i = 0; i < m; ++i) bound = ids[i] + 1 > bound ? ids[i] + 1 : bound;
    // counting sort by id; universes are visited in order, so each id's members come out in universe order
    std::vector<int64_t> cnt(bound + 1, 0);
    for (int64_t i = 0; i < m; ++i) ++cnt[ids[i] + 1];
    int64_t groups = 0;
    for (int64_t g = 1; g <= bound; ++g) groups += cnt[g] > 0;
    const int64_t need = 8 * groups + 5 * m;   // J id, EMPTY_SET, MARK, (J universe) * k, ADDITEMS
    *n_out = need;
    if (!out) return PT_OK;
    if (cap < need) return PT_EINVAL;
    std::vector<int64_t> start(bound + 1, 0);
    for (int64_t g = 0; g < bound; ++g) start[g + 1] = start[g] + cnt[g + 1];
    std::vector<int64_t> fill(start.begin(), start.end() - 1);
    std::vector<int32_t> member(m);
    std::vector<int64_t> order;   // ids in order of first appearance
    order.reserve(groups);
    for (int64_t u = 0; u < n; ++u)
        for (int64_t i = off[u]; i < off[u + 1]; ++i) {
            const int64_t g = ids[i];
            if (fill[g] == start[g]) order.push_back(g);
            member[fill[g]++] = static_cast<int32_t>(uids[u]);
        }
    uint8_t *p = out;
    for (int64_t g : order) {
        p = put_int(p, g);
        *p++ = 0x8f;   // EMPTY_SET
        *p++ = '(';
        for (int64_t j = start[g]; j < start[g + 1]; ++j) p = put_int(p, member[j]);
        *p++ = 0x90;   // ADDITEMS
    }
    return PT_OK;
}
