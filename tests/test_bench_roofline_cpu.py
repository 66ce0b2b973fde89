"""bench.py's universe-line roofline helpers on the CPU: chain_floor (the dependent-chain floor of a universe step,
+ VALU issue from rocprofv3 counts) and residency (which universes ran beside a profiled one, from the profile
words 7 and 63 that pt_universe_set_profile returns)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_chain_floor_grows_with_rounds_and_counts_valu():
    small = bench.chain_floor(0, 200, 32, 100)
    big = bench.chain_floor(0, 200, 96, 300)
    # 1024-thread workgroup, 32-lane groups for D = 200: 32 positives per round of phase A
    assert small["shape"]["lanes"] == 32 and small["shape"]["lane_groups"] == 32
    assert small["rounds_a"] == 1 and big["rounds_a"] == 3
    assert big["latency_cycles"] > small["latency_cycles"]
    assert small["floor_cycles"] == small["latency_cycles"]
    with_valu = bench.chain_floor(0, 200, 32, 100, valu_per_step=8000)
    # 8,000 wave-instructions over 4 SIMDs at 2 cycles each
    assert with_valu["valu_issue_cycles"] == 4000.0
    assert with_valu["floor_cycles"] == small["latency_cycles"] + 4000.0


def _profile_rows(entries):
    """Synthetic pt_universe_set_profile rows: (start tick, duration ticks, XCD, SE, CU) per universe."""
    pr = np.zeros((len(entries), 64), dtype=np.uint64)
    for i, (start, dur, xcc, se, cu) in enumerate(entries):
        pr[i, 7] = (np.uint64(start) << np.uint64(32)) | np.uint64(dur)
        pr[i, 63] = (np.uint64(xcc) << np.uint64(32)) | np.uint64((se << 13) | (cu << 8))
    return pr.astype(np.float64)


def test_residency_counts_overlap_weighted_neighbours():
    pr = _profile_rows([
        (100, 1000, 2, 1, 3),    # the universe asked about
        (100, 1000, 2, 1, 3),    # same CU, whole time
        (600, 1000, 2, 0, 0),    # same XCD, half its time
        (100, 1000, 5, 1, 3),    # another XCD (same SE / CU ids)
        (5000, 100, 2, 1, 3),    # same CU, after it ended
    ])
    r = bench.residency(pr, 0)
    assert r["xcd"] == 2
    assert abs(r["same_cu"] - 1.0) < 1e-12
    assert abs(r["same_xcd"] - 1.5) < 1e-12
    assert r["universes_per_xcd"][2] == 4 and r["universes_per_xcd"][5] == 1


def test_residency_of_an_unprofiled_universe_is_none():
    pr = _profile_rows([(0, 0, 0, 0, 0)])
    assert bench.residency(pr, 0) is None
