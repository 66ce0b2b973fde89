// Sanitizer driver (ASan + UBSan, or TSan) for the HOST side of libputranse_hip: the reader, the universe
// construction (single and the multi-threaded pt_universe_build_many), the host ranking (pt_rank_queries on
// worker threads), the Base.so-compatible global context (importTrainFiles ... getParallelUniverse /
// swapHelpers / resetUniverse, importTestFiles, testHead / testTail / test_link_prediction, getTestBatch) and
// the CPU oracle's multi-threaded loops (oracle_train_loop_mt, oracle_train_step_mt). No GPU call is made.
// Every multi-threaded result is compared with its one-thread form. Built and run by
// `make -C openke-putranse_amd san SAN=address|thread` (tests/test_native_cpu.py::test_host_sanitizers).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "putranse.h"
extern "C" {
#include "oracle.h"
}

static int failures = 0;
#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                           \
        }                                                                         \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s KG_DIR/\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[1];
    // ---- reader + universe construction: pt_universe_build_many (8 threads) == pt_universe_build
    pt_graph *g = nullptr;
    CHECK(pt_graph_load(dir.c_str(), &g) == 0);
    const int64_t n = 48;
    std::vector<int64_t> seeds(n), tcs(n);
    std::vector<float> bals(n);
    for (int64_t i = 0; i < n; ++i) {
        seeds[i] = 4 + i;
        tcs[i] = 200 + 37 * i;
        bals[i] = 0.25f + 0.005f * (float)i;
    }
    std::vector<pt_universe *> many(n, nullptr);
    CHECK(pt_universe_build_many(g, n, seeds.data(), 8, tcs.data(), bals.data(), 8, many.data()) == 0);
    for (int64_t i = 0; i < n; ++i) {
        pt_universe *one = nullptr;
        CHECK(pt_universe_build(g, seeds[i], 8, tcs[i], bals[i], &one) == 0);
        const int64_t E = pt_universe_ent_total(one), R = pt_universe_rel_total(one);
        CHECK(E == pt_universe_ent_total(many[i]) && R == pt_universe_rel_total(many[i]));
        CHECK(pt_universe_train_total(one) == pt_universe_train_total(many[i]));
        std::vector<int64_t> e1(E), r1(R), e2(E), r2(R);
        pt_universe_remaps(one, e1.data(), r1.data());
        pt_universe_remaps(many[i], e2.data(), r2.data());
        CHECK(e1 == e2 && r1 == r2);
        std::vector<uint64_t> s1(8), s2(8);
        pt_universe_seeds(one, s1.data());
        pt_universe_seeds(many[i], s2.data());
        CHECK(s1 == s2);
        pt_universe_free(one);
        pt_universe_free(many[i]);
    }
    // ---- host ranking on 8 worker threads == 1 worker
    const int64_t E = pt_graph_ent_total(g), N = pt_graph_train_total(g);
    std::vector<int64_t> th(N), tt(N), tr(N);
    CHECK(pt_graph_triples(g, th.data(), tt.data(), tr.data()) == 0);
    pt_known *k = nullptr;
    CHECK(pt_known_create(th.data(), tt.data(), tr.data(), N, &k) == 0);
    const int64_t q = 64;
    std::vector<float> con((size_t)(q * E));
    uint64_t x = 12345;
    for (auto &v : con) {
        x = x * 6364136223846793005ULL + 1442695040888963407ULL;
        v = (float)(x >> 40) / (float)(1 << 24);
    }
    for (int side = 0; side < 2; ++side) {
        std::vector<int64_t> raw1(q), f1(q), raw8(q), f8(q);
        CHECK(pt_rank_queries(k, E, th.data(), tt.data(), tr.data(), q, side, con.data(), raw1.data(), f1.data(), 1) == 0);
        CHECK(pt_rank_queries(k, E, th.data(), tt.data(), tr.data(), q, side, con.data(), raw8.data(), f8.data(), 8) == 0);
        CHECK(raw1 == raw8 && f1 == f8);
        std::vector<int64_t> off(q + 1);
        CHECK(pt_known_partners(k, side, q, side ? th.data() : tt.data(), tr.data(), off.data(), nullptr) == 0);
        std::vector<int64_t> part((size_t)std::max<int64_t>(off[q], 1));
        CHECK(pt_known_partners(k, side, q, side ? th.data() : tt.data(), tr.data(), off.data(), part.data()) == 0);
    }
    pt_known_free(k);
    // ---- the Base.so-compatible global context (host paths)
    std::vector<char> path(dir.begin(), dir.end());
    path.push_back(0);
    setInPath(path.data());
    setRandomSeed(4);
    randReset();
    importTrainFiles();
    CHECK(pt_legacy_import_status() == 0);
    CHECK(getEntityTotal() == E && getTrainTotal() == N);
    for (int u = 0; u < 3; ++u) {
        setRandomSeed(4 + u);
        randReset();
        getParallelUniverse(300 + 100 * u, 0.3f);
        const int64_t Eu = getEntityTotalUniverse(), Ru = getRelationTotalUniverse();
        CHECK(Eu > 0 && Ru > 0 && getTrainTotalUniverse() > 0);
        std::vector<int64_t> em(Eu), rm(Ru);
        getEntityRemapping(em.data());
        getRelationRemapping(rm.data());
        swapHelpers();
        CHECK(getEntityTotal() == Eu);
        resetUniverse();
        CHECK(getEntityTotal() == E);
    }
    importTestFiles();
    CHECK(pt_legacy_import_status() == 0);
    const int64_t nt = getTestTotal();
    CHECK(nt > 0);
    {
        std::vector<int64_t> ph(nt), pt_(nt), pr(nt), nh(nt), nt_(nt), nr(nt);
        getTestBatch(ph.data(), pt_.data(), pr.data(), nh.data(), nt_.data(), nr.data());
    }
    initTest();
    std::vector<int64_t> bh(E), bt(E), br(E);
    std::vector<float> sc(E);
    for (int64_t i = 0; i < nt; ++i) {
        getHeadBatch(bh.data(), bt.data(), br.data());
        for (int64_t j = 0; j < E; ++j) sc[j] = con[(size_t)((i % q) * E + j)];
        testHead(sc.data(), i, 0);
        getTailBatch(bh.data(), bt.data(), br.data());
        testTail(sc.data(), i, 0);
    }
    test_link_prediction(0);
    CHECK(std::isfinite(getTestLinkMRR(0)) && getTestLinkHit10(0) >= 0.f && getTestLinkHit10(0) <= 1.f);
    validInit();
    for (int64_t i = 0; i < getValidTotal(); ++i) {
        getValidHeadBatch(bh.data(), bt.data(), br.data());
        validHead(sc.data(), i);
        getValidTailBatch(bh.data(), bt.data(), br.data());
        validTail(sc.data(), i);
    }
    CHECK(std::isfinite(getValidHit10()));
    // ---- CPU oracle: the multi-threaded training loop == the one-thread loop, bit for bit
    okg *og = okg_load(dir.c_str());
    CHECK(og != nullptr);
    const int64_t D = 16, OE = okg_ent_total(og), OR = okg_rel_total(og);
    for (int model = 0; model < 2; ++model) {
        std::vector<float> t1[6], t8[6];
        const int64_t rows[6] = {OE, OR, OR, OE, OR, OR};
        for (int a = 0; a < 6; ++a) {
            t1[a].assign((size_t)(rows[a] * D), 0.f);
            for (size_t j = 0; a < 3 && j < t1[a].size(); ++j) {
                x = x * 6364136223846793005ULL + 1442695040888963407ULL;
                t1[a][j] = (float)((int64_t)(x >> 41) - (1LL << 22)) / (float)(1 << 24);
            }
            t8[a] = t1[a];
        }
        orand_t r1, r8;
        orand_seed(&r1, 4);
        orand_seed(&r8, 4);
        std::vector<uint64_t> s1(8), s8(8);
        oracle_rand_reset(&r1, 8, s1.data());
        oracle_rand_reset(&r8, 8, s8.data());
        std::vector<float> l8(6);
        oracle_train_loop(og, s1.data(), 8, 64, 3, 1, 1, model, 1, 1, 1, 0.05f, 2.f, D, t1[0].data(), t1[1].data(),
                          t1[2].data(), t1[3].data(), t1[4].data(), t1[5].data(), 6);
        oracle_train_loop_mt(og, s8.data(), 8, 64, 3, 1, 1, model, 1, 1, 1, 0.05f, 2.f, D, t8[0].data(), t8[1].data(),
                             t8[2].data(), t8[3].data(), t8[4].data(), t8[5].data(), 6, 8, l8.data());
        for (int a = 0; a < 6; ++a) CHECK(std::memcmp(t1[a].data(), t8[a].data(), t1[a].size() * 4) == 0);
        CHECK(s1 == s8);
    }
    okg_free(og);
    pt_graph_free(g);
    std::printf("san_driver: %s (%d failed checks)\n", failures ? "FAIL" : "ok", failures);
    return failures ? 1 : 0;
}
