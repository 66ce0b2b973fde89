"""Benchmark: training triples/s (positive + negative slots) of the fused TransE/TransH step on MI355X.

Default workload = BASELINE.json configs[1] (C2): TransE on FB15K237-shaped synthetic data, dim 200,
batch 2000, 25 negatives per positive, L2 norm, SGD (alpha 1.0, margin 5), bern + filter sampling,
8 emulated sampler threads. One "step" = Trainer.train_one_step's work on one batch: in-kernel sampling
of 2000 positives x (1 + 25) slots, NegativeSampling + MarginLoss forward, backward, SGD update of the
touched rows. Inputs (graph, tables) are resident in HBM before timing starts.

  python bench.py [--gpus N --steps K --warmup W]

N > 1: bench.py runs as one rank per GPU; started without a torch.distributed environment it launches the N
ranks itself (torch.distributed.run, 127.0.0.1) before touching the GPU and relays rank 0's line.

C2 is a single model, so N > 1 runs N independent replicas (one per GPU, "replicas only", weak
scaling, no collective in the data path); value = slots of all ranks / max-over-ranks time.
Prints ONE JSON line on rank 0 with roofline (live HIP-event kernel timing, per-kernel counted bytes from
the committed PMC summary) and cpu_baseline (the oracle's C restatement on the host's cores, at most 16
threads, timed on a bounded sample of the same workload, rank 0, N = 1); the pu_c3 field (C3 universes)
carries its own cpu_baseline.
"""
import argparse
import ctypes
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(HERE, "openke-putranse_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(PKG, "tools"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

WORKLOADS = {
    # name: (shape, model, dim, p_norm, opt, lr, margin, batch_size, neg, bern, filter)
    "c2": ("fb15k237", "TransE", 200, 2, "sgd", 1.0, 5.0, 2000, 25, 1, 1),
    "c1": ("wn18", "TransE", 50, 1, "sgd", 1.0, 4.0, 100, 1, 0, 1),
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, Chip-level parameters)


def algorithmic_bytes_per_slot(model, opt, dim):
    """index reads (3 x int64) + one read and one write of every row a slot touches."""
    base = {("TransE", "sgd"): 24, ("TransE", "adagrad"): 48, ("TransH", "sgd"): 32, ("TransH", "adagrad"): 64}
    return base[(model, opt)] * dim + 24


def dist_setup():
    """One process per GPU over RCCL (backend "nccl"). PT_BENCH_BACKEND=gloo runs the same multi-rank logic
    over gloo with ranks sharing the visible GPUs (rank -> GPU local_rank % device_count): a rehearsal of the
    N > 1 path on a one-GPU box, not a measurement."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1:
        import torch.distributed as dist
        backend = os.environ.get("PT_BENCH_BACKEND", "nccl")
        dev = local % torch.cuda.device_count()
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return ws, rank, local


def spawn_ranks(n):
    """`bench.py --gpus N` (N > 1) started without a torch.distributed environment: start N fresh ranks under
    torch.distributed.run (one process per GPU, 127.0.0.1 rendezvous) with the same arguments, relay their output
    and return their exit status. Runs before anything in this process touches the GPU (the parent only counts
    devices), and starts the ranks as children: a GPU-initialised process is never replaced."""
    import socket
    import subprocess
    backend = os.environ.get("PT_BENCH_BACKEND", "nccl")
    if backend == "nccl":
        have = torch.cuda.device_count()
        if have < n:
            print("bench.py: --gpus %d needs %d visible GPUs, found %d" % (n, n, have), file=sys.stderr)
            return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    p = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    line = None
    for ln in p.stdout.splitlines():
        print(ln, flush=True)
        if ln.startswith("{"):
            line = ln
    if p.returncode != 0:
        return p.returncode
    try:
        got = json.loads(line)["n_gpus"] if line else None
    except ValueError:
        got = None
    if got != n:
        print("bench.py: --gpus %d but the ranks reported n_gpus %s" % (n, got), file=sys.stderr)
        return 3
    return 0


def barrier(ws):
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()


def all_reduce(t, op):
    """In-place all_reduce of a device tensor (through host memory when the backend is gloo)."""
    import torch.distributed as dist
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=op)
    else:
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)


def all_gather_padded(t, ws):
    """Every rank's 1-D tensor `t` (lengths may differ) on every rank, as a list in rank order: one all_gather of
    the lengths, one of the payloads padded to the longest (through host memory when the backend is gloo)."""
    import torch.distributed as dist
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    ns = [torch.zeros_like(n) for _ in range(ws)]
    gloo = dist.get_backend() != "nccl"
    if gloo:
        ns = [x.cpu() for x in ns]
        dist.all_gather(ns, n.cpu())
    else:
        dist.all_gather(ns, n)
    lens = [int(x.item()) for x in ns]
    m = max(max(lens), 1)
    pad = torch.zeros(m, dtype=t.dtype, device=t.device)
    pad[:t.numel()] = t
    outs = [torch.zeros_like(pad) for _ in range(ws)]
    if gloo:
        outs = [x.cpu() for x in outs]
        dist.all_gather(outs, pad.cpu())
        outs = [x.to(t.device) for x in outs]
    else:
        dist.all_gather(outs, pad)
    return [o[:k] for o, k in zip(outs, lens)]


def gather_universes(unis, ws):
    """Every rank's trained universes (tables, remaps, dims) on every rank - the input of an N = 1 recomputation of
    the link prediction: one all_gather each of the universes' sizes, their tables (float32) and their remaps
    (int64). Returns the union as a list of universe dicts (rank order, then each rank's order)."""
    dev = unis[0]["ent"].device if unis else (torch.device("cuda", torch.cuda.current_device())
                                              if torch.cuda.is_available() else torch.device("cpu"))
    meta = torch.tensor([[u["ent"].shape[0], u["rel"].shape[0], u["dim"], int(u["nv"] is not None)] for u in unis],
                        dtype=torch.int64, device=dev).reshape(-1)
    flat = [u[k].reshape(-1) for u in unis for k in ("ent", "rel", "nv") if u[k] is not None]
    tabs = torch.cat(flat) if flat else torch.zeros(0, device=dev)
    maps = torch.from_numpy(np.concatenate([np.concatenate([u["em"], u["rm"]]) for u in unis])
                            if unis else np.zeros(0, np.int64)).to(dev)
    metas, tabss, mapss = (all_gather_padded(x, ws) for x in (meta, tabs, maps))
    out = []
    for mt, tb, mp in zip(metas, tabss, mapss):
        mt = mt.reshape(-1, 4).cpu().numpy()
        mp = mp.cpu().numpy()
        ot = om = 0
        for E, R, D, has_nv in mt:
            u = {"dim": int(D)}
            for k, rows in (("ent", E), ("rel", R), ("nv", R if has_nv else 0)):
                u[k] = tb[ot:ot + rows * D].reshape(int(rows), int(D)) if rows else None
                ot += rows * D
            u["em"], u["rm"] = mp[om:om + E].copy(), mp[om + E:om + E + R].copy()
            om += E + R
            out.append(u)
    return out


def rank_digest(ranks):
    """SHA-1 of the raw / filtered head and tail rank vectors (int64, query order)."""
    import hashlib
    m = hashlib.sha1()
    for r in ranks:
        m.update(np.ascontiguousarray(r, dtype=np.int64).tobytes())
    return m.hexdigest()


def cpu_workers():
    """Host threads for the CPU baseline: the cores this process may run on, at most 16 (a one-GPU box's
    CPU share; the reference's sampler uses 8 pthreads, Base.cpp:266-310)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(path, wl, seconds=12.0):
    """The CPU restatement (oracle/oracle.c: the reference's sampler + the step in reference order) on
    `cpu_workers()` threads - sampler slices and the per-slot / per-row phases in parallel, bit-identical
    to its single-thread form - over a bounded sample of the same workload."""
    sys.path.insert(0, HERE)
    import oracle
    shape, model, dim, p, opt, lr, margin, bs, neg, bern, filt = wl
    workers = cpu_workers()
    kg = oracle.KG.load(path)
    st = oracle.GlibcRand(4).rand_reset(8)
    rng = np.random.default_rng(0)
    bound = np.sqrt(6.0 / (kg.ent_total + dim))
    ent = rng.uniform(-bound, bound, (kg.ent_total, dim)).astype(np.float32)
    rel = rng.uniform(-bound, bound, (kg.rel_total, dim)).astype(np.float32)
    nv = rng.uniform(-bound, bound, (kg.rel_total, dim)).astype(np.float32) if model == "TransH" else None
    accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv))
    oracle.train_loop(kg, st, 8, bs, neg, bern, filt, model, p, True, opt, lr, margin, (ent, rel, nv), accs, 1,
                      workers=workers)
    steps, slots, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        slots += oracle.train_loop(kg, st, 8, bs, neg, bern, filt, model, p, True, opt, lr, margin,
                                   (ent, rel, nv), accs, 1, workers=workers)
        steps += 1
    el = time.perf_counter() - t0
    return {"value": slots / el, "unit": "triples/s", "cores": workers, "kind": "port",
            "sample": "%d steps of the same workload (batch %d x (1+%d), dim %d) on the same synthetic graph, "
                      "oracle/oracle.c on %d threads (sampler slices + per-slot / per-row phases), %.1f s"
                      % (steps, bs, neg, dim, workers, el)}


# PuTransE workloads (BASELINE.json configs[2..4]); ranges from the reference's experiments
# (static_experiment_PuTransE_on_WN18.py:67-88, static_experiment_PuTransH_on_WN18.py:70-79,
# incremental_experiment_PuTransE_on_WikidataEvolve.py:173-182)
PU_WORKLOADS = {
    # name: shape, universes, model, dim (int or (lo, hi) per-universe draw), p, tc range, margin range, lp
    "c3": ("wn18", 512, "TransE", (20, 100), 1, (500, 2000), (1, 4), False),
    "c4": ("wikidata", 1024, "TransE", 200, 1, (500, 1500), (1, 5), True),
    "c5": ("fb15k", 256, "TransH", 20, 1, (500, 2000), (1, 4), False),
}


# Chain roofline of a universe (the universe lines' bound: one universe is one workgroup's dependent step chain,
# its working set cache-resident, so HBM bandwidth does not describe it). Latency constants from
# /opt/skills/guides/MI355X_MICROARCH.md "Per-instruction cycle constants": global_load L2-hit latency ~180-225 cyc,
# ds_read latency ~50 cyc, v_fma dependent latency ~4 cyc; a DPP / permlane step of a lane-group reduction is
# taken as 8 cyc (an op plus its data hazard), a workgroup barrier as 50 cyc.
CHAIN_L2, CHAIN_LDS, CHAIN_DPP, CHAIN_BAR = 200, 50, 8, 50


def universe_shape(mid, D):
    """(G, VEC, KCH, NT, RB) of a universe row of dim D - pick_universe_shape / universe_class_threads /
    universe_run's RB (csrc/universes.hip, universes.h, universes_kern.h)."""
    vec = 4 if D % 4 == 0 else 1
    chunks = -(-D // vec)
    per_lane = 2 if vec == 4 else (8 if mid == 0 else 4)
    G = 2
    while G < 64 and G * per_lane < chunks:
        G *= 2
    kch = 1
    while G * kch < chunks:
        kch *= 2
    if (2 if vec == 4 else 4) <= G <= (8 if vec == 4 else 16):
        kch = -(-chunks // G)
    floats = vec * kch
    nt = 1024 if mid == 0 and floats <= 8 else 512
    rb = 1 if floats >= 16 else ((1 if (mid == 1 or nt > 512) else 2) if floats > 4 else (2 if nt > 512 else 4))
    return G, vec, kch, nt, rb


def chain_floor(mid, D, bs, rows_per_step, valu_per_step=None):
    """Cycles per step a universe's step chain cannot go below (universes_kern.h universe_run), by phase:
    phase A, ceil(bs / lane groups) rounds of one positive per lane group, each round the dependent chain
      LDS (batch) -> L2 (positive rows; wide rows also the first negative's) -> reduction (normalizations)
      -> reduction (positive score) -> [narrow rows: LDS + L2 (negative row) + reduction] -> reduction (negative
      score) -> 4 LDS round trips (the contribution links: negative, relation flag, head, tail);
    phase B, ceil(rows / (lane groups x rows per group)) rounds, each
      LDS (work list) -> LDS (list head) -> L2 (row, Adagrad state, first contribution) -> reduction (the
      normalize Jacobian's dot product);
    two workgroup barriers per step; a reduction over G lanes = log2(G) DPP steps + one op. With
    `valu_per_step` (VALU wave-instructions per step of the universe, rocprofv3 SQ_INSTS_VALU of it alone) the
    issue time of those instructions on the CU's 4 SIMDs at 2 cycles each (SIMD-32 throughput) is added: the
    floor then is latency chain + VALU issue."""
    G, vec, kch, nt, rb = universe_shape(mid, D)
    gpb = nt // G
    red = CHAIN_DPP * (G.bit_length() - 1) + CHAIN_DPP
    wide = G >= 32 and mid == 0
    rounds_a = -(-max(bs, 1) // gpb)
    a_round = CHAIN_LDS + CHAIN_L2 + 3 * red + (0 if wide else CHAIN_LDS + CHAIN_L2 + red) + 4 * CHAIN_LDS
    rounds_b = -(-max(int(round(rows_per_step)), 1) // (gpb * rb))
    b_round = 2 * CHAIN_LDS + CHAIN_L2 + red
    lat = rounds_a * a_round + rounds_b * b_round + 2 * CHAIN_BAR
    out = {"shape": {"lanes": G, "vec": vec, "chunks_per_lane": kch, "threads": nt, "lane_groups": gpb,
                     "rows_per_group": rb},
           "rounds_a": rounds_a, "a_round_cycles": a_round, "rounds_b": rounds_b, "b_round_cycles": b_round,
           "barriers_cycles": 2 * CHAIN_BAR, "latency_cycles": lat,
           "constants": {"l2_hit": CHAIN_L2, "lds": CHAIN_LDS, "dpp_step": CHAIN_DPP, "barrier": CHAIN_BAR}}
    if valu_per_step is not None:
        out["valu_issue_cycles"] = 2.0 * valu_per_step / 4.0
        out["floor_cycles"] = lat + out["valu_issue_cycles"]
    else:
        out["floor_cycles"] = float(lat)
    return out


def universe_draws(k, tc_range=(500, 2000), margin_range=(1, 4), seed0=4):
    """Python-RNG hyperparameters of universe k exactly as Parallel_Universe_Config draws them
    (:157-161, :210-236): randrange(tc), uniform(balance), randrange(margin), randrange(epochs),
    uniform(lr) rounded to 3 digits."""
    import random
    rs = random.Random(seed0 + k)
    tc = rs.randrange(*tc_range)
    bal = round(rs.uniform(0.25, 0.5), 2)
    margin = rs.randrange(*margin_range)
    epochs = rs.randrange(50, 200)
    lr = round(rs.uniform(0.001, 0.1), 3)
    return tc, bal, margin, epochs, lr


def _xavier(rng, rows, dim):
    b = np.sqrt(6.0 / (rows + dim))
    return rng.uniform(-b, b, (rows, dim)).astype(np.float32)


def team_info(row):
    """A profiled universe's team (pt_universe_set_profile words 60-61; None: one workgroup)."""
    w = int(row[60]) >> 32
    if w <= 1:
        return None
    steps = max(float(row[3]), 1.0)
    return {"width": w, "one_xcd": bool(int(row[60]) & 1), "barrier_cycles_per_step": float(row[61]) / steps}


def residency(pr, i):
    """Where universe i of a profiled set ran against the others (pt_universe_set_profile word 7: start / duration on
    the 100 MHz wall clock; word 63: XCD and HW_REG_HW_ID - SE, SH, CU fields): the time-averaged count of other
    universes running beside it on its CU and on its XCD (the XCD's L2), and the set's average per XCD."""
    w7 = pr[:, 7].astype(np.uint64)
    start = (w7 >> np.uint64(32)).astype(np.float64)
    dur = (w7 & np.uint64(0xffffffff)).astype(np.float64)
    w63 = pr[:, 63].astype(np.uint64)
    xcc = (w63 >> np.uint64(32)).astype(np.int64)
    hw = (w63 & np.uint64(0xffffffff)).astype(np.int64)
    cu = xcc * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15)
    if dur[i] <= 0:
        return None
    ov = np.clip(np.minimum(start + dur, start[i] + dur[i]) - np.maximum(start, start[i]), 0, None) / dur[i]
    ov[i] = 0.0
    return {"xcd": int(xcc[i]), "same_cu": float(ov[cu == cu[i]].sum()), "same_xcd": float(ov[xcc == xcc[i]].sum()),
            "universes_per_xcd": [int((xcc == x).sum()) for x in range(8)],
            "note": "time-averaged other universes beside the longest one on its CU / its XCD (profile words 7, 63)"}


def chain_profile(L, us, reset, idx, time_set, mid, name, prof_on, rel_of=None, target=None):
    """One extra (untimed) training of the set with the per-universe cycle counters on. The roofline universe is
    `target` - the (bs, dim, ent, steps) of the set's longest universe by the placement cost model, the one
    `--longest-only` trains and tools_gpu/pmc_chain.sh counts - its measured cycles per step in the set against
    chain_floor, with VALU issue in the floor when profiles/pmc_<name>_chain.json holds its rocprofv3 counts on this
    library build; `set_longest` is the universe that ran longest in this training (which one that is varies with
    where the universes land: DESIGN.md section 6), against its floor without VALU unless it is the target.
    Phase-B rows: a team universe counts member 0's (profile word 62); a one-workgroup universe's are the expected
    distinct rows of a step - bs * (2 + neg) entity draws over E rows and bs relation draws over R (rel_of[(bs, D,
    E)]), E (1 - exp(-n / E)) each (uniform draws: an estimate; the kernel keeps no counter)."""
    from openke import _native
    if not prof_on:
        _native.check(L.pt_universe_set_profiling(us, 1))
    time_set(us, reset, idx, 1, 0)
    pr = np.zeros(64 * len(idx), dtype=np.uint64)
    _native.check(L.pt_universe_set_profile(us, pr.ctypes.data))
    if not prof_on:
        _native.check(L.pt_universe_set_profiling(us, 0))
    pr = pr.reshape(-1, 64).astype(np.float64)
    span = pr[:, :3].sum(axis=1)
    pmc, _ = load_pmc("%s_chain" % name)

    def entry(i):
        steps = max(pr[i, 3], 1.0)
        bs, D, E = int(pr[i, 4]), int(pr[i, 5]), int(pr[i, 6])
        R = (rel_of or {}).get((bs, D, E), 0)
        rows_estimated = pr[i, 62] == 0
        if rows_estimated:
            rows = E * (1.0 - np.exp(-bs * 3.0 / max(E, 1))) + (R * (1.0 - np.exp(-bs / R)) if R else 0.0)
        else:
            rows = pr[i, 62] / steps
        key = {"bs": bs, "dim": D, "ent": E, "steps": int(steps)}
        valu = pmc["valu_per_step"] if pmc and pmc.get("longest") == key else None
        fl = chain_floor(mid, D, bs, rows, valu)
        achieved = span[i] / steps
        return {"achieved": achieved, "floor": fl["floor_cycles"], "frac": fl["floor_cycles"] / achieved,
                "universe": dict(key, rows_per_step=rows, rows_estimated=bool(rows_estimated), cycles=span[i],
                                 **{"ms_at_2.4GHz": span[i] / 2.4e6},
                                 cycles_per_step={"presample": pr[i, 0] / steps, "phase_a": pr[i, 1] / steps,
                                                  "phase_b": pr[i, 2] / steps}),
                "floor_model": fl, "valu_counted": valu is not None, "team": team_info(pr[i]),
                "residency": residency(pr, i)}
    i_long = int(np.argmax(span))
    hit = [j for j in range(len(pr)) if target is not None and
           (int(pr[j, 4]), int(pr[j, 5]), int(pr[j, 6]), int(pr[j, 3])) == target]
    i_t = hit[0] if hit else i_long
    out = entry(i_t)
    out["unit"] = "cycles/step"
    out["roofline_universe"] = ("the set's longest by the placement cost model (the universe pmc_chain.sh counts)"
                                if hit else "the universe that ran longest")
    out["longest_universe"] = out.pop("universe")
    lg = entry(i_long)
    out["set_longest"] = {"universe": lg["universe"], "achieved": lg["achieved"], "floor": lg["floor"],
                          "frac": lg["frac"], "valu_counted": lg["valu_counted"], "residency": lg["residency"]}
    return out


def run_universes(args, ws, rank, dev, name="c3", cpu=True, per_gpu=False, check_lp=False):
    """PuTransE / PuTransH universes placed over ranks by LPT (place_universes; no collective in training), Adagrad,
    neg 1, bern 0, filter 0, nbatches 20, 8 sampler threads. One step = every universe's full training
    run (all its epochs) in one persistent launch. C4 adds link prediction over the test split: each
    rank MINs its universes' scores into the key rows, one RCCL all_reduce(MIN), GPU ranking."""
    import synth_kg
    from openke import _native
    L = _native.lib()
    shape, n_univ, model, dim_spec, p_norm, tc_range, margin_range, do_lp = PU_WORKLOADS[name]
    if getattr(args, "universes", 0):   # --universes: the reference experiment's own count (e.g. 6,000)
        n_univ = args.universes
    if getattr(args, "dim", 0):         # --dim: one fixed dim (the reference experiment's 20)
        dim_spec = args.dim
    if per_gpu:   # weak scaling: the workload's universe count on EVERY GPU (universes 4+k continue the seeds)
        n_univ *= ws
        do_lp = False
    path = synth_kg.ensure_dataset(os.path.join(args.data_dir, "rank%d" % rank), shape)
    g = ctypes.c_void_p()
    _native.check(L.pt_graph_load(path.encode(), ctypes.byref(g)))
    from openke.config.Parallel_Universe_Config import place_universes, universe_cost
    all_draws = [universe_draws(k, tc_range, margin_range) for k in range(n_univ)]
    if isinstance(dim_spec, tuple):
        all_dims = [int(np.random.default_rng(1000 + k).integers(dim_spec[0], dim_spec[1] + 1)) for k in range(n_univ)]
    else:
        all_dims = [dim_spec] * n_univ
    # LPT placement over ranks on the drawn sizes (tc approximates the universe's triple count)
    owners = place_universes({k: universe_cost(all_draws[k][3], all_draws[k][0], all_dims[k]) for k in range(n_univ)},
                             ws)
    own = [k for k in range(n_univ) if owners[k] == rank]
    draws = [all_draws[k] for k in own]
    dims = [all_dims[k] for k in own]
    seeds = np.array([4 + k for k in own], dtype=np.int64)
    tcs = np.array([d[0] for d in draws], dtype=np.int64)
    bals = np.array([d[1] for d in draws], dtype=np.float32)
    handles = (ctypes.c_void_p * max(len(own), 1))()
    t0 = time.perf_counter()
    _native.check(L.pt_universe_build_many(g, len(own), seeds.ctypes.data, 8, tcs.ctypes.data, bals.ctypes.data, 0,
                                           handles))
    build_s = time.perf_counter() - t0
    mid = 0 if model == "TransE" else 1
    jobs, keep, unis = [], [], []
    slots_step, bytes_step = 0, 0
    for i, k in enumerate(own):
        h = handles[i]
        E, R, N = L.pt_universe_ent_total(h), L.pt_universe_rel_total(h), L.pt_universe_train_total(h)
        D = dims[i]
        rng = np.random.default_rng(k)
        ent = torch.from_numpy(_xavier(rng, E, D)).to(dev)
        rel = torch.from_numpy(_xavier(rng, R, D)).to(dev)
        nv = torch.from_numpy(_xavier(rng, R, D)).to(dev) if mid == 1 else None
        accs = [torch.zeros_like(x) if x is not None else None for x in (ent, rel, nv)]
        st = np.zeros(8, dtype=np.uint64)
        _native.check(L.pt_universe_seeds(h, st.ctypes.data))
        tc, bal, margin, epochs, lr = draws[i]
        bs = N // 20
        j = _native.UniverseJob()
        j.graph = L.pt_universe_graph(h)
        j.seeds = st.ctypes.data
        j.threads, j.batch_size, j.epochs, j.nbatches, j.neg = 8, bs, epochs, 20, 1
        j.lr, j.margin = lr, margin
        j.ent, j.rel, j.normv = ent.data_ptr(), rel.data_ptr(), nv.data_ptr() if nv is not None else None
        j.ent_acc, j.rel_acc = accs[0].data_ptr(), accs[1].data_ptr()
        j.norm_acc = accs[2].data_ptr() if accs[2] is not None else None
        j.dim = D
        jobs.append(j)
        keep.append((st, accs))
        em = np.zeros(max(E, 1), dtype=np.int64)
        rm = np.zeros(max(R, 1), dtype=np.int64)
        _native.check(L.pt_universe_remaps(h, em.ctypes.data, rm.ctypes.data))
        unis.append({"ent": ent, "rel": rel, "nv": nv, "em": em[:E], "rm": rm[:R], "dim": D,
                     "init": tuple(x.clone() if x is not None else None for x in (ent, rel, nv))})
        slots = epochs * 20 * bs * 2
        slots_step += slots
        bytes_step += slots * algorithmic_bytes_per_slot(model, "adagrad", D)
    prof_on = os.environ.get("PT_UNI_PROF") == "1"
    has_reset = hasattr(L, "pt_universe_set_reset")

    def make_set(idx):
        """A universe set of jobs[idx]; returns (set handle, reset function restoring every table, Adagrad
        state and sampler stream to its initial value - each timed run trains from the same start)."""
        arr = (_native.UniverseJob * max(len(idx), 1))(*[jobs[i] for i in idx])
        us = ctypes.c_void_p()
        _native.check(L.pt_universe_set_create(arr, len(idx), mid, p_norm, 1, _native.PT_ADAGRAD, 0, 0,
                                               ctypes.byref(us)))
        if prof_on:
            _native.check(L.pt_universe_set_profiling(us, 1))

        def reset():
            for i in idx:
                u = unis[i]
                for live, init in zip((u["ent"], u["rel"], u["nv"]), u["init"]):
                    if live is not None:
                        live.copy_(init)
                for a in keep[i][1]:
                    if a is not None:
                        a.zero_()
            if has_reset:   # (an older build under A/B lacks it: its streams continue instead)
                _native.check(L.pt_universe_set_reset(us))
        return us, reset

    def time_set(us, reset, idx, steps, warmup):
        """Seconds of `steps` trainings of the set (after `warmup` untimed ones), each from the initial state:
        the reset outside the timed region, barrier + synchronize on both sides of every timed training."""
        total_epochs = sum(int(jobs[i].epochs) for i in idx)
        losses = torch.zeros(max(total_epochs, 1), device=dev)
        stream = _native.stream()
        el = 0.0
        for s_ in range(warmup + steps):
            reset()
            torch.cuda.synchronize()
            barrier(ws)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            _native.check(L.pt_universe_set_train(us, _native.ptr(losses), stream))
            torch.cuda.synchronize()
            barrier(ws)
            if s_ >= warmup:
                el += time.perf_counter() - t0
        assert torch.isfinite(losses).all(), "non-finite universe loss"
        return el

    def launch_times(us):
        """The set's concurrent class launches in its last training (pt_universe_set_launch_times): per launch
        start / end (ms after the first start) and universes, and their overlap = summed launch time over the span
        (the launch count when all run side by side from the start, 1.0 when they run one after another)."""
        if not hasattr(L, "pt_universe_set_launch_times"):
            return None
        n = ctypes.c_int64(0)
        _native.check(L.pt_universe_set_launch_times(us, 0, None, ctypes.byref(n)))
        if n.value == 0:
            return None
        buf = np.zeros(3 * n.value, dtype=np.float32)
        _native.check(L.pt_universe_set_launch_times(us, n.value, buf.ctypes.data, ctypes.byref(n)))
        rows = buf.reshape(-1, 3)
        span = float(rows[:, 1].max() - rows[:, 0].min())
        return {"launches": [[round(float(a), 3), round(float(b), 3), int(c)] for a, b, c in rows],
                "span_ms": span, "overlap": float((rows[:, 1] - rows[:, 0]).sum()) / max(span, 1e-9),
                "latest_start_ms": float(rows[:, 0].max()),
                "note": "[start ms, end ms, universes] per class launch of the last timed training (HIP events on "
                        "each launch's stream); overlap = summed launch time / span"}

    every = list(range(len(jobs)))
    if getattr(args, "longest_only", False) and jobs:
        # the set's longest universe alone (by the placement cost model): its chain, e.g. under rocprofv3 --pmc
        i_long = max(every, key=lambda i: universe_cost(int(jobs[i].epochs), int(jobs[i].batch_size) * 20,
                                                        int(jobs[i].dim)))
        every = [i_long]
        slots_step = int(jobs[i_long].epochs) * 20 * int(jobs[i_long].batch_size) * 2
        bytes_step = slots_step * algorithmic_bytes_per_slot(model, "adagrad", int(jobs[i_long].dim))
    uset, reset = make_set(every)
    el = time_set(uset, reset, every, args.c3_steps, args.c3_warmup)
    class_launches = launch_times(uset)
    rel_of = {(int(jobs[i].batch_size), int(jobs[i].dim), int(unis[i]["ent"].shape[0])): int(unis[i]["rel"].shape[0])
              for i in every}
    # the roofline universe: the longest by the placement cost model (the one --longest-only and pmc_chain.sh take)
    i_m = max(every, key=lambda i: universe_cost(int(jobs[i].epochs), int(jobs[i].batch_size) * 20,
                                                 int(jobs[i].dim))) if every else None
    target = (int(jobs[i_m].batch_size), int(jobs[i_m].dim), int(unis[i_m]["ent"].shape[0]),
              int(jobs[i_m].epochs) * 20) if every else None
    chain = chain_profile(L, uset, reset, every, time_set, mid, name, prof_on, rel_of, target) if every else None
    tot = torch.tensor([el, float(slots_step), float(bytes_step)], dtype=torch.float64, device=dev)
    if ws > 1:
        import torch.distributed as dist
        mx = tot[:1].clone()
        all_reduce(mx, dist.ReduceOp.MAX)
        all_reduce(tot, dist.ReduceOp.SUM)
        el = float(mx.item())
    slots_all, bytes_all = float(tot[1].item()), float(tot[2].item())
    longest = None
    if prof_on:
        prof = np.zeros(64 * max(len(jobs), 1), dtype=np.uint64)
        _native.check(L.pt_universe_set_profile(uset, prof.ctypes.data))
        prof = prof.reshape(-1, 64)
        # the set's schedule: each universe's start (100 MHz wall clock, low 32 bits) and duration, in ms
        w_start = (prof[:, 7] >> np.uint64(32)).astype(np.int64)
        w_start = ((w_start - w_start.min()) % (1 << 32)).astype(np.float64) * 1e-5
        w_dur = (prof[:, 7] & np.uint64(0xffffffff)).astype(np.float64) * 1e-5
        prof = prof.astype(np.float64)
        span = prof[:, :3].sum(axis=1)
        il = int(np.argmax(span))
        print("universe-prof schedule: last end %.2f ms after the first start; the longest universe starts at %.2f ms "
              "and runs %.2f ms; universes starting after 1 ms: %d" % ((w_start + w_dur).max(), w_start[il], w_dur[il],
                                                                       int((w_start > 1.0).sum())), file=sys.stderr)
        longest = float(span.max())
        for i in np.argsort(-span)[:6]:   # the longest universes (cycles of the last run)
            steps = max(prof[i, 3], 1)
            print("universe-prof span %.1f Mcyc steps %d bs %d D %d E %d  cycles/step: presample %.0f"
                  "  A %.0f  B %.0f" % (span[i] / 1e6, steps, prof[i, 4], prof[i, 5], prof[i, 6],
                                       prof[i, 0] / steps, prof[i, 1] / steps, prof[i, 2] / steps), file=sys.stderr)
        if os.environ.get("PT_UNI_PROF_DUMP"):   # every universe's phase cycles + its job (time-model fits)
            np.savez(os.environ["PT_UNI_PROF_DUMP"], prof=prof, dims=np.array([int(j.dim) for j in jobs]),
                     bs=np.array([int(j.batch_size) for j in jobs]), epochs=np.array([int(j.epochs) for j in jobs]),
                     E=np.array([u["ent"].shape[0] for u in unis]), R=np.array([u["rel"].shape[0] for u in unis]),
                     run_s=el / args.c3_steps,
                     start_ms=w_start, dur_ms=w_dur)
        tot_p = prof[:, :3].sum(axis=0) / max(prof[:, 3].sum(), 1)
        print("universe-prof all: cycles/step presample %.0f A %.0f B %.0f" % tuple(tot_p), file=sys.stderr)
        print("universe-prof longest universe: %.1f Mcycles (%.1f ms at 2.4 GHz); run %.1f ms" %
              (span.max() / 1e6, span.max() / 2.4e6, el * 1e3 / args.c3_steps), file=sys.stderr)
    det_s = None
    if args.deterministic_timing and ws == 1:
        # the reference-order mode (bit-identical to the oracle) on the same set, one training from the start
        _native.check(L.pt_universe_set_deterministic(uset, 1))
        det_s = time_set(uset, reset, every, 1, 0)
        _native.check(L.pt_universe_set_deterministic(uset, 0))
    _native.check(L.pt_universe_set_free(uset))
    placement = None
    if args.place_world > 1 and ws == 1:
        # one GPU, the per-rank critical path of a place_world-way job: each rank's LPT share (place_universes,
        # as Parallel_Universe_Config places a wave) trained alone, from the initial state
        pw = args.place_world
        po = place_universes({k: universe_cost(all_draws[k][3], all_draws[k][0], all_dims[k]) for k in own}, pw)
        shares, spans, teams_r = [], [], []
        for r in range(pw):
            idx = [i for i, k in enumerate(own) if po[k] == r]
            us, rs = make_set(idx)
            if not prof_on:
                _native.check(L.pt_universe_set_profiling(us, 1))
            shares.append(time_set(us, rs, idx, args.c3_steps, 1) / args.c3_steps)
            pr = np.zeros(64 * max(len(idx), 1), dtype=np.uint64)
            _native.check(L.pt_universe_set_profile(us, pr.ctypes.data))
            prr = pr.reshape(-1, 64)
            span_r = prr[:, :3].astype(np.float64).sum(axis=1)
            if os.environ.get("PT_UNI_PROF_DUMP") and idx:   # the share's universes (time-model fits)
                np.savez(os.environ["PT_UNI_PROF_DUMP"].replace(".npz", "_share%d.npz" % r), prof=prr,
                         dims=np.array([int(jobs[i].dim) for i in idx]), bs=np.array([int(jobs[i].batch_size) for i in idx]),
                         epochs=np.array([int(jobs[i].epochs) for i in idx]),
                         E=np.array([unis[i]["ent"].shape[0] for i in idx]),
                         R=np.array([unis[i]["rel"].shape[0] for i in idx]))
            spans.append(float(span_r.max()) if idx else 0.0)
            if idx:
                il = int(np.argmax(span_r))
                st = max(float(prr[il, 3]), 1.0)
                t0w = min(int(w) >> 32 for w in prr[:, 7])
                # the share's longest universes: [universe, cycles, XCD, start (10 ns wall-clock ticks)]
                top = [[int(j), float(span_r[j]), int(prr[j, 63]) >> 32, (int(prr[j, 7]) >> 32) - t0w]
                       for j in np.argsort(-span_r)[:6]]
                teams_r.append({"team": team_info(prr[il].astype(np.float64)), "top_spans": top,
                                "residency": residency(prr.astype(np.float64), il), "cycles_per_step": {
                                    "presample": float(prr[il, 0]) / st, "phase_a": float(prr[il, 1]) / st,
                                    "phase_b": float(prr[il, 2]) / st}})
            _native.check(L.pt_universe_set_free(us))
        placement = {"world": pw, "universes_per_rank": [sum(1 for k in own if po[k] == r) for r in range(pw)],
                     "share_s": shares, "max_share_s": max(shares), "rank0_share_s": shares[0],
                     "full_set_s": el / args.c3_steps, "max_share_over_full": max(shares) / (el / args.c3_steps),
                     "longest_universe_cycles_per_share": spans, "longest_universe_per_share": teams_r,
                     "note": "one GPU: rank r's LPT share of a %d-way placement trained alone (the N = %d per-rank "
                             "critical path); longest-universe spans in shader-clock cycles" % (pw, pw)}
    for i in range(len(own)):
        L.pt_universe_free(handles[i])
    achieved = bytes_all * args.c3_steps / el / 1e9 / max(ws, 1)
    out = {"workload": "%s Pu%s %s-shaped, %d universes, D=%s, p%d, tc~U[%d,%d), epochs~U[50,200), Adagrad, neg 1, "
                       "nbatches 20" % (name.upper(), model, shape, n_univ,
                                        "U{%d..%d}" % dim_spec if isinstance(dim_spec, tuple) else dim_spec, p_norm,
                                        tc_range[0], tc_range[1]),
           "value": slots_all * args.c3_steps / el, "unit": "triples/s", "scaling": "weak" if per_gpu else "strong",
           "steps": args.c3_steps, "warmup": args.c3_warmup, "s_per_step": el / args.c3_steps,
           "universes_per_gpu": len(own), "host_universe_build_s": build_s,
           "note_runs": "every timed run trains every universe from its initial tables, Adagrad state and sampler "
                        "streams (restored before the run, outside the timed region)",
           "roofline": dict(chain or {}, bound="chain", algorithmic_GBps_per_gpu=achieved,
                            note="the set ends with its longest universe, one workgroup's dependent step chain: achieved "
                                 "= that universe's measured shader cycles per step (pt_universe_set_profiling, one "
                                 "extra untimed training), floor = chain_floor's model of it (bench.py: L2 / LDS round "
                                 "trips, lane-group reductions, barriers, + VALU issue when its rocprofv3 counters are "
                                 "committed for this build), frac = floor / achieved; the floor takes L2 hits, which a "
                                 "universe alone gets (hit rate 0.997) and a full set does not (C4: 0.27, "
                                 "profiles/r06_c4_l2.txt). algorithmic_GBps_per_gpu: SURVEY 8(d) bytes per wall second")}
    if class_launches is not None:
        out["class_launches"] = class_launches
    if det_s is not None:
        out["deterministic_s_per_step"] = det_s
        out["deterministic_triples_per_s"] = slots_step / det_s
    if placement is not None:
        out["placement"] = placement
    if longest is not None:
        out["longest_universe_cycles"] = longest
    if do_lp:
        out["link_prediction"] = lp = universe_link_prediction(L, path, unis, mid, p_norm, ws, dev)
        if check_lp and ws > 1:
            # the N = 1 recomputation: every rank's trained universes gathered, rank 0 scores and ranks all of them
            # alone (no collective) - the distributed ranks must be bit-identical (MIN is exact)
            t0 = time.perf_counter()
            allu = gather_universes(unis, ws)
            lp["gather_universes_s"] = time.perf_counter() - t0
            if rank == 0:
                ref = universe_link_prediction(L, path, allu, mid, p_norm, 1, dev)
                lp["n1_universes"] = len(allu)
                lp["n1_rank_digest"] = ref["rank_digest"]
                lp["n1_mrr_mr_hit10_hit3_hit1"] = ref["mrr_mr_hit10_hit3_hit1"]
                lp["digest_match"] = ref["rank_digest"] == lp["rank_digest"]
            del allu
    L.pt_graph_free(g)
    if cpu and ws == 1 and rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = universe_cpu_baseline(path, name, args.cpu_seconds, getattr(args, "dim", 0),
                                                    getattr(args, "universes", 0))
    return out


def run_dropin(args, ws, rank, dev, name="c3"):
    """The drop-in universe path timed as the reference's experiments drive it
    (experiments/static_experiment_PuTransE_on_WN18.py:40-91): TrainDataLoader(nbatches 20, threads 8, normal
    sampling, bern 0, filter 0, neg 1) and TestDataLoader on the same synthetic graph, Parallel_Universe_Config
    with the workload's hyperparameter ranges, train_parallel_universes(n) with valid_steps = n / 4 (a divisor of
    n: validation, early-stopping bookkeeping and best-model checkpoints at 4 points, as the experiment's
    valid_steps 100 does over its 6,000 universes), then run_link_prediction() for C4. The universes are those
    of the kernel-only line (same seeds 4 + k, draws, dims). Reported: wall seconds of each call and the
    breakdown Parallel_Universe_Config records (draws, native construction, torch modules, H2D, the training
    launch, commits, validation + checkpoints)."""
    import shutil
    import synth_kg
    from openke.config import Parallel_Universe_Config
    from openke.data import TestDataLoader, TrainDataLoader
    from openke.module.model import TransE, TransH
    shape, n_univ, model, dim_spec, p_norm, tc_range, margin_range, do_lp = PU_WORKLOADS[name]
    if getattr(args, "universes", 0):
        n_univ = args.universes
    if getattr(args, "dim", 0):
        dim_spec = args.dim
    do_lp = do_lp or getattr(args, "link_prediction", False)
    valid_steps = args.valid_steps if getattr(args, "valid_steps", 0) else max(n_univ // 4, 1)
    path = synth_kg.ensure_dataset(os.path.join(args.data_dir, "rank%d" % rank), shape)
    t0 = time.perf_counter()
    train_dl = TrainDataLoader(in_path=path, nbatches=20, threads=8, sampling_mode="normal", bern_flag=0,
                               filter_flag=0, neg_ent=1, neg_rel=0, random_seed=4)
    test_dl = TestDataLoader(train_dl.in_path, "link")
    ck = tempfile.mkdtemp(prefix="pu_dropin_") + os.sep
    cfg = Parallel_Universe_Config(
        training_identifier="bench_%s" % name, train_dataloader=train_dl, test_dataloader=test_dl,
        initial_num_universes=None, min_margin=margin_range[0], max_margin=margin_range[1], min_lr=0.001,
        max_lr=0.1, min_num_epochs=50, max_num_epochs=200, min_triple_constraint=tc_range[0],
        max_triple_constraint=tc_range[1], min_balance=0.25, max_balance=0.5,
        embedding_model=TransE if model == "TransE" else TransH,
        embedding_model_param={"dim": dim_spec, "p_norm": p_norm, "norm_flag": 1},
        checkpoint_dir=ck, valid_steps=valid_steps, save_steps=10000, training_setting="static",
        incremental_strategy=None)
    setup_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    barrier(ws)
    t0 = time.perf_counter()
    cfg.train_parallel_universes(n_univ)
    torch.cuda.synchronize()
    barrier(ws)
    train_s = time.perf_counter() - t0
    out = {"universes": n_univ, "setup_s": setup_s, "train_parallel_universes_s": train_s, "wave_size": cfg.wave_size(),
           "valid_steps": cfg.valid_steps, "universes_committed": cfg.next_universe_id,
           "breakdown_s": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in cfg.last_train_timing.items()}}
    if do_lp:
        torch.cuda.synchronize()
        barrier(ws)
        t0 = time.perf_counter()
        met = cfg.run_link_prediction()
        torch.cuda.synchronize()
        barrier(ws)
        out["run_link_prediction_s"] = time.perf_counter() - t0
        out["mrr_mr_hit10_hit3_hit1"] = [float(x) for x in met]
    shutil.rmtree(ck, ignore_errors=True)
    return out


def universe_cpu_baseline(path, name, seconds, dim_override=0, n_override=0):
    """The CPU restatement training whole universes of the same workload on `cpu_workers()` threads (one
    universe per thread at a time, taken in id order; the reference trains them one after another on one
    process, Parallel_Universe_Config.py:316-327): construction + epochs x 20 Adagrad steps each, new
    universes started until `seconds` have elapsed, the clock stopped when the last one finishes."""
    import threading
    sys.path.insert(0, HERE)
    import oracle
    shape, n_univ, model, dim_spec, p_norm, tc_range, margin_range, _ = PU_WORKLOADS[name]
    if dim_override:
        dim_spec = dim_override
    if n_override:
        n_univ = n_override
    workers = cpu_workers()
    kg = oracle.KG.load(path)
    lock = threading.Lock()
    state = {"next": 0, "slots": 0, "done": 0}
    t0 = time.perf_counter()

    def work():
        while True:
            with lock:
                k = state["next"]
                if k >= n_univ or time.perf_counter() - t0 >= seconds:
                    return
                state["next"] += 1
            tc, bal, margin, epochs, lr = universe_draws(k, tc_range, margin_range)
            D = int(np.random.default_rng(1000 + k).integers(dim_spec[0], dim_spec[1] + 1)) \
                if isinstance(dim_spec, tuple) else dim_spec
            rng_c = oracle.GlibcRand(4 + k)
            st = rng_c.rand_reset(8)
            ug, _, _ = kg.universe(rng_c, tc, bal)
            bs = ug.train_total // 20
            rng = np.random.default_rng(k)
            ent = _xavier(rng, ug.ent_total, D)
            rel = _xavier(rng, ug.rel_total, D)
            nv = _xavier(rng, ug.rel_total, D) if model == "TransH" else None
            accs = (np.zeros_like(ent), np.zeros_like(rel), None if nv is None else np.zeros_like(nv))
            n = oracle.train_loop(ug, st, 8, bs, 1, 0, 0, model, p_norm, True, "adagrad", lr, margin,
                                  (ent, rel, nv), accs, epochs * 20)
            with lock:
                state["slots"] += n
                state["done"] += 1

    ths = [threading.Thread(target=work) for _ in range(workers)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    return {"value": state["slots"] / el, "unit": "triples/s", "cores": workers, "kind": "port",
            "sample": "%d whole universes (construction + epochs x 20 Adagrad steps) of the same workload, "
                      "oracle/oracle.c, one universe per thread on %d threads, %.1f s" % (state["done"], workers, el)}


def universe_link_prediction(L, path, unis, mid, p_norm, ws, dev):
    """PuTransE link prediction of the test split over the trained universes (global energy
    estimation, Parallel_Universe_Config.py:446-642): per rank pt_lp_min_scores of its universes into
    the key rows, RCCL all_reduce(MIN), pt_rank_rows, pt_lp_metrics. Timed end to end on the device."""
    from openke import _native
    from openke.config.Parallel_Universe_Config import lp_pair_array, lp_pairs_all
    E = sum(1 for _ in open(os.path.join(path, "entity2id.txt")))
    trip = {f: np.loadtxt(os.path.join(path, f), dtype=np.int64, ndmin=2) for f in
            ("train2id.txt", "valid2id.txt", "test2id.txt")}
    allt = np.concatenate(list(trip.values()))
    known = ctypes.c_void_p()
    ah, at, ar = (np.ascontiguousarray(allt[:, c]) for c in range(3))
    _native.check(L.pt_known_create(ah.ctypes.data, at.ctypes.data, ar.ctypes.data, len(ah), ctypes.byref(known)))
    th, tt, tr = (np.ascontiguousarray(trip["test2id.txt"][:, c]) for c in range(3))
    n = len(th)
    keys = {}
    q_row = [np.zeros(n, np.int64), np.zeros(n, np.int64)]
    for q in range(n):
        for side, anchor in ((0, int(tt[q])), (1, int(th[q]))):
            q_row[side][q] = keys.setdefault((side, anchor, int(tr[q])), len(keys))
    ks = np.array([k[0] for k in keys], np.int64)
    ka = np.array([k[1] for k in keys], np.int64)
    kr = np.array([k[2] for k in keys], np.int64)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rows = torch.full((len(keys), E), float("inf"), device=dev)
    tup = torch.full((len(keys),), float("inf"), device=dev)
    lp_us = []
    # every universe's local->global entity map in one device array (one copy)
    moff = np.cumsum([0] + [len(u["em"]) for u in unis])
    dremaps = torch.from_numpy(np.concatenate([u["em"] for u in unis]) if unis else np.zeros(1, np.int64)).to(dev)
    for slot, u in enumerate(unis):
        U = _native.LpUniverse()
        U.ent, U.rel = u["ent"].data_ptr(), u["rel"].data_ptr()
        U.normv = u["nv"].data_ptr() if u["nv"] is not None else None
        U.ent_total, U.rel_total, U.dim = u["ent"].shape[0], u["rel"].shape[0], u["dim"]
        U.d_ent_remap = dremaps.data_ptr() + 8 * int(moff[slot])
        lp_us.append(U)
    pair_arr, arr_p = lp_pair_array([lp_pairs_all([u["em"] for u in unis], [u["rm"] for u in unis], ka, kr, ks)])
    if len(pair_arr):
        arr_u = (_native.LpUniverse * len(lp_us))(*lp_us)
        _native.check(L.pt_lp_min_scores(arr_u, len(lp_us), mid, p_norm, 1, arr_p, len(pair_arr), E, _native.ptr(rows),
                                         _native.ptr(tup), _native.stream()))
    torch.cuda.synchronize()
    t_score = time.perf_counter() - t0
    if ws > 1:
        import torch.distributed as dist
        all_reduce(rows, dist.ReduceOp.MIN)
        all_reduce(tup, dist.ReduceOp.MIN)
    torch.cuda.synchronize()
    t_comb = time.perf_counter() - t0 - t_score
    ranks = []
    for side, anchor, truth in ((0, tt, th), (1, th, tt)):
        off = np.zeros(n + 1, np.int64)
        _native.check(L.pt_known_partners(known, side, n, anchor.ctypes.data, tr.ctypes.data, off.ctypes.data, None))
        part = np.zeros(max(int(off[-1]), 1), np.int64)
        _native.check(L.pt_known_partners(known, side, n, anchor.ctypes.data, tr.ctypes.data, off.ctypes.data,
                                          part.ctypes.data))
        d_row = torch.from_numpy(q_row[side]).to(dev)
        d_truth = torch.from_numpy(truth).to(dev)
        d_off, d_part = torch.from_numpy(off).to(dev), torch.from_numpy(part).to(dev)
        raw = torch.zeros(n, dtype=torch.int64, device=dev)
        filt = torch.zeros(n, dtype=torch.int64, device=dev)
        _native.check(L.pt_rank_rows(_native.ptr(rows), E, _native.ptr(d_row), _native.ptr(d_truth), None,
                                     _native.ptr(d_off), _native.ptr(d_part), n, _native.ptr(raw), _native.ptr(filt),
                                     _native.stream()))
        ranks += [raw.cpu().numpy(), filt.cpu().numpy()]
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    met = np.zeros(10, dtype=np.float32)
    _native.check(L.pt_lp_metrics(ranks[0].ctypes.data, ranks[1].ctypes.data, ranks[2].ctypes.data,
                                  ranks[3].ctypes.data, n, met.ctypes.data))
    L.pt_known_free(known)
    # scored (pair, candidate) cells: every local entity of the pair's universe (k_lp_scan_t: one lane per entity,
    # the pair's base row uniform across the wave; per cell and dim one LDS read and ~3 VALU lane-operations)
    ent_of = np.array([len(u["em"]) for u in unis], dtype=np.int64)
    cells = int(ent_of[pair_arr[:, 1]].sum()) if len(pair_arr) else 0
    dim_of = np.array([u["dim"] for u in unis], dtype=np.int64)
    cell_dims = int((ent_of[pair_arr[:, 1]] * dim_of[pair_arr[:, 1]]).sum()) if len(pair_arr) else 0
    return {"queries": int(n), "keys": len(keys), "pairs_this_rank": len(pair_arr), "seconds": el,
            "rank_digest": rank_digest(ranks),
            "scored_cells": cells, "scored_cell_dims": cell_dims,
            "score_s": t_score, "min_combine_s": t_comb, "rank_s": el - t_score - t_comb,
            "mrr_mr_hit10_hit3_hit1": [float(x) for x in met[:5]],
            "note": "universe scoring 4D+4 B per (key, universe entity); ranking 4 B per (query, entity)"}


def library_sha256():
    """sha256 of the library this process loaded (the product build unless tools_gpu/ablib.py swapped it)."""
    import hashlib
    from openke import _native
    return hashlib.sha256(open(_native.LIB_PATH, "rb").read()).hexdigest()


def load_pmc(tag):
    """The committed rocprofv3 --pmc summary profiles/pmc_<tag>.json when it was taken on THIS library build
    (its lib_sha256 equals the loaded library's), else None: counter evidence is never borrowed from another
    build. Returns (summary or None, its digest)."""
    f = os.path.join(HERE, "profiles", "pmc_%s.json" % tag)
    if not os.path.exists(f):
        return None, None
    try:
        rec = json.load(open(f))
    except Exception:
        return None, None
    sha = rec.get("lib_sha256")
    return (rec if sha and sha == library_sha256() else None), sha


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS) + sorted(PU_WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--repeats", type=int, default=5, help="timed repeats of the K-step run (value = median)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--data-dir", default=os.path.join(tempfile.gettempdir(), "putranse_bench"))
    ap.add_argument("--no-c3", action="store_true", help="skip the PuTransE universe workload (C3) field")
    ap.add_argument("--c3-steps", type=int, default=2)
    ap.add_argument("--c3-warmup", type=int, default=1)
    ap.add_argument("--place-world", type=int, default=0,
                    help="universe workloads on one GPU: also time each rank's LPT share of a PLACE_WORLD-way job")
    ap.add_argument("--deterministic-timing", type=int, default=1,
                    help="also time the reference-order (deterministic) mode (1: yes)")
    ap.add_argument("--step-apply", type=int, default=0,
                    help="C2 / C1: 1 = the fused step + apply kernel where it applies (opt-in, measured slower), 0 = "
                         "the step + apply pair (default; pt_trainer_set_step_apply)")
    ap.add_argument("--universes", type=int, default=0,
                    help="universe workloads: this many universes instead of the config's (the reference experiment "
                         "trains 6,000: experiments/static_experiment_PuTransE_on_WN18.py:84-91)")
    ap.add_argument("--dim", type=int, default=0,
                    help="universe workloads: one fixed embedding dim instead of the config's (the reference experiment: 20)")
    ap.add_argument("--link-prediction", action="store_true",
                    help="universe workloads: the drop-in leg ends with run_link_prediction() (as the reference "
                         "experiment does; C4 always does)")
    ap.add_argument("--valid-steps", type=int, default=0,
                    help="drop-in leg: validate every this many universes (default: a quarter of the universes; the "
                         "reference experiment uses 100)")
    ap.add_argument("--no-ref-scale", action="store_true",
                    help="default line: skip the pu_c3_ref6000 field (6,000 universes, dim 20, strong scaling)")
    ap.add_argument("--slot-scale", type=int, default=-1,
                    help="C2 / C1: 1 = slot-scale mode (per-slot records + positive base rows instead of contribution "
                         "rows; pt_trainer_set_slot_scale), 0 = contribution rows, -1 = the library's default")
    ap.add_argument("--team-width", type=int, default=0,
                    help="universe workloads: widest team per universe when a GPU holds fewer universes than CUs "
                         "(pt_set_universe_team_width: 1, 2 or 4; 0 = the library default)")
    ap.add_argument("--longest-only", action="store_true",
                    help="universe workloads: train only the set's longest universe (its chain alone)")
    ap.add_argument("--no-dropin", action="store_true",
                    help="universe workloads: skip the drop-in Parallel_Universe_Config timing")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, check the world size against --gpus, print it and stop (no GPU work)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        print("bench.py: WORLD_SIZE %s differs from --gpus %d" % (os.environ.get("WORLD_SIZE", "1"), args.gpus),
              file=sys.stderr)
        sys.exit(3)
    if args.launch_check:
        ws = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        if ws > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            t = torch.ones(1)
            dist.all_reduce(t)
            ws_seen = int(t.item())
            dist.destroy_process_group()
        else:
            ws_seen = 1
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": ws_seen, "world_size_env": ws}), flush=True)
        return

    ws, rank, local = dist_setup()
    if args.team_width:
        from openke import _native
        _native.check(_native.lib().pt_set_universe_team_width(args.team_width))
    if args.workload in PU_WORKLOADS:
        dev = torch.device("cuda", torch.cuda.current_device())
        args.c3_steps, args.c3_warmup = args.steps, args.warmup
        c3 = run_universes(args, ws, rank, dev, args.workload)
        dropin = None if args.no_dropin else run_dropin(args, ws, rank, dev, args.workload)
        if rank == 0:
            rec = {"metric": "training triples/sec (pos+neg)", "value": c3["value"], "unit": "triples/s",
                   "n_gpus": ws, "steps": args.steps, "warmup": args.warmup, "ms_per_step": c3["s_per_step"] * 1e3,
                   "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
                   "data": "synthetic %s-shaped graph (tools/synth_kg.py, seed 0), xavier-uniform tables" %
                           PU_WORKLOADS[args.workload][0],
                   "config": {"workload": c3["workload"], "parallelism": "universes placed by LPT over %d ranks" % ws},
                   "roofline": c3["roofline"], "universes_per_gpu": c3["universes_per_gpu"]}
            if "link_prediction" in c3:
                rec["link_prediction"] = c3["link_prediction"]
            if dropin is not None:
                rec["dropin"] = dropin
            for k in ("placement", "class_launches", "deterministic_s_per_step", "deterministic_triples_per_s", "longest_universe_cycles",
                      "note_runs", "host_universe_build_s"):
                if k in c3:
                    rec[k] = c3[k]
            if "cpu_baseline" in c3:
                rec["cpu_baseline"] = c3["cpu_baseline"]
            print(json.dumps(rec), flush=True)
        if ws > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    wl = WORKLOADS[args.workload]
    shape, model, dim, p, opt, lr, margin, bs, neg, bern, filt = wl

    import synth_kg
    from openke import _native
    from openke.config import Trainer
    from openke.data import TrainDataLoader
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE, TransH
    from openke.module.strategy import NegativeSampling

    data_dir = os.path.join(args.data_dir, "rank%d" % rank)
    path = synth_kg.ensure_dataset(data_dir, shape)
    dl = TrainDataLoader(in_path=path, batch_size=bs, threads=8, sampling_mode="normal", bern_flag=bern,
                         filter_flag=filt, neg_ent=neg, neg_rel=0, random_seed=4)
    torch.manual_seed(rank)
    cls = TransE if model == "TransE" else TransH
    kge = cls(ent_tot=dl.get_ent_tot(), rel_tot=dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=True)
    ns = NegativeSampling(model=kge, loss=MarginLoss(margin=margin), batch_size=bs)
    tr = Trainer(model=ns, data_loader=dl, train_times=0, alpha=lr, use_gpu=True, opt_method=opt)
    tr.run()   # moves the tables to HBM and builds the native trainer; no steps
    L = _native.lib()
    _native.check(L.pt_trainer_set_step_apply(tr._native, args.step_apply))
    if args.slot_scale >= 0:
        _native.check(L.pt_trainer_set_slot_scale(tr._native, args.slot_scale))
    sampler = dl.device_sampler()
    dev = torch.device("cuda", torch.cuda.current_device())
    seq = bs * (1 + neg)

    # warmup (also instantiates the hipGraph of `steps` replayed steps)
    wl_losses = torch.zeros(max(args.warmup, 1), device=dev)
    if args.warmup > 0:
        _native.check(L.pt_trainer_run(tr._native, sampler, bs, neg, bern, filt, args.warmup,
                                       _native.ptr(wl_losses), _native.stream()))
    losses = torch.zeros(args.steps, device=dev)
    # capture the timed graph outside the timed region: run it once untimed after warmup
    _native.check(L.pt_trainer_run(tr._native, sampler, bs, neg, bern, filt, args.steps, _native.ptr(losses),
                                   _native.stream()))
    torch.cuda.synchronize()

    # the K-step replay timed `repeats` times (each bracketed by barrier + synchronize, max over ranks); value is
    # the median (box-to-box and run-to-run spread shows in the min / max alongside)
    runs = []
    for _ in range(max(args.repeats, 1)):
        barrier(ws)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _native.check(L.pt_trainer_run(tr._native, sampler, bs, neg, bern, filt, args.steps, _native.ptr(losses),
                                       _native.stream()))
        torch.cuda.synchronize()
        barrier(ws)
        el = time.perf_counter() - t0
        if ws > 1:
            import torch.distributed as dist
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            all_reduce(tt, dist.ReduceOp.MAX)
            el = float(tt.item())
        runs.append(el)
    el = float(np.median(runs))
    det_ms = None
    if args.deterministic_timing:
        # the reference-order mode (Trainer(deterministic=True): bit-identical to the oracle), same K steps
        _native.check(L.pt_trainer_set_deterministic(tr._native, 1))
        dl_ = torch.zeros(args.steps, device=dev)
        _native.check(L.pt_trainer_run(tr._native, sampler, bs, neg, bern, filt, args.steps, _native.ptr(dl_),
                                       _native.stream()))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _native.check(L.pt_trainer_run(tr._native, sampler, bs, neg, bern, filt, args.steps, _native.ptr(dl_),
                                       _native.stream()))
        torch.cuda.synchronize()
        det_ms = (time.perf_counter() - t0) * 1e3 / args.steps
        _native.check(L.pt_trainer_set_deterministic(tr._native, 0))
    loss_last = float(losses[-1].item())
    assert np.isfinite(loss_last), "non-finite loss"

    # live kernel timing with HIP events on the launch stream (roofline of the fused step): the same
    # per-step kernels launched one by one with an event pair around each; per-chunk sampling/scan
    # launches amortised over the steps they serve
    ms4 = (ctypes.c_float * 4)()
    n_t = min(256, args.steps)   # the timed run's chunking (sampling launches cover up to 256 steps)
    tl = torch.zeros(n_t, device=dev)
    _native.check(L.pt_trainer_run_timed(tr._native, sampler, bs, neg, bern, filt, n_t, _native.ptr(tl), ms4,
                                         _native.stream()))
    # the sampling kernels of the path the library took for this chunking (pt_trainer_last_path)
    spath = L.pt_trainer_last_path(tr._native)
    fused_sa = bool(L.pt_trainer_step_apply(tr._native))
    slot_sc = bool(L.pt_trainer_slot_scale(tr._native)) if hasattr(L, "pt_trainer_slot_scale") else False
    step_names = (["k_step_apply", "k_loss_calls"] if fused_sa else
                  ["k_step_csr", "k_apply_buf"] if spath != _native.PT_PATH_SAMPLED else ["k_step_sampled", "k_apply"])
    names = list(_native.PATH_KERNELS.get(spath, ("sampling", "bucket scan"))) + step_names
    per_kernel = {n: float(v) for n, v in zip(names, ms4) if n and v > 0}
    bytes_step = algorithmic_bytes_per_slot(model, opt, dim) * seq
    step_kernel_s = sum(per_kernel.values()) * 1e-3
    achieved = bytes_step / step_kernel_s / 1e9
    pmc, pmc_sha = load_pmc(args.workload)
    traffic = pmc.get("bytes_per_step") if pmc else None
    counted = pmc.get("bytes_per_step_by_kernel") if pmc else None
    kernel_detail = {}
    for kname, ms in per_kernel.items():
        b = next((v for k, v in counted.items() if kname in k), None) if counted else None
        kernel_detail[kname] = {"ms": ms, "counted_bytes": b,
                                "counted_TBps": None if b is None or ms <= 0 else b / (ms * 1e-3) / 1e12}
    # gradient rows of the corrupted entities: stored by the step, read by apply (slot-scale mode: an 8-byte record
    # per slot and three base rows per positive instead)
    contrib_rt = 2 * (bs * neg * 8 + bs * 3 * dim * 4) if slot_sc else 2 * bs * neg * dim * 4

    c3 = None if args.no_c3 else run_universes(args, ws, rank, dev, "c3", cpu=True)
    if c3 is not None and ws == 1 and not args.no_dropin:
        # the drop-in universe path on the same C3 set, as experiments/static_experiment_PuTransE_on_WN18.py
        # drives it (Parallel_Universe_Config.train_parallel_universes), beside the kernel-only time above
        c3["dropin"] = run_dropin(args, ws, rank, dev, "c3")
        c3["dropin"]["over_kernel_only"] = c3["dropin"]["train_parallel_universes_s"] / c3["s_per_step"]
    # universe weak scaling (512 universes per GPU, no collective): at N = 1 it is the strong line
    c3w = None if args.no_c3 or ws == 1 else run_universes(args, ws, rank, dev, "c3", cpu=False, per_gpu=True)
    # the reference experiment's own scale (experiments/static_experiment_PuTransE_on_WN18.py:43-91: 6,000
    # universes, dim 20), kernel-only, strong scaling over the ranks: enough universes per GPU at N = 8 (750) that
    # the set is throughput-bound, not bound by its longest universe as the 512-universe C3 set is
    c3r = None
    if not args.no_c3 and not args.no_ref_scale:
        import copy as _copy
        a2 = _copy.copy(args)
        a2.universes, a2.dim, a2.place_world, a2.deterministic_timing = 6000, 20, 0, 0
        c3r = run_universes(a2, ws, rank, dev, "c3", cpu=False)
    # N > 1: the one collective of the path (north_star: RCCL over xGMI for the score combine at link prediction) in
    # the default line - C4's 1,024 universes placed over the ranks by LPT, each rank's universes MIN-combined into
    # the key rows, one all_reduce(MIN), GPU ranking; rank 0 checks the ranks against an N = 1 recomputation
    c4lp = None
    if ws > 1 and not args.no_c3:
        import copy as _copy
        a4 = _copy.copy(args)
        a4.universes, a4.dim, a4.place_world, a4.deterministic_timing = 0, 0, 0, 0
        c4lp = run_universes(a4, ws, rank, dev, "c4", cpu=False, check_lp=True)
    if rank != 0:
        if ws > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    value = args.steps * seq * ws / el
    rec = {
        "metric": "training triples/sec (pos+neg)",
        "value": value,
        "unit": "triples/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el * 1e3 / args.steps,
        "repeats": len(runs),
        "ms_per_step_runs": [r * 1e3 / args.steps for r in runs],
        "value_best": args.steps * seq * ws / min(runs),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic %s-shaped graph (tools/synth_kg.py, seed 0), xavier-uniform tables" % shape,
        "config": {"workload": "%s %s %s-shaped dim %d p%d %s lr %g margin %g batch %d neg %d bern %d filter %d "
                               "threads 8" % (args.workload.upper(), model, shape, dim, p, opt, lr, margin, bs, neg,
                                              bern, filt),
                   "global_batch": seq * ws, "slots_per_step_per_gpu": seq,
                   "parallelism": "replicas%d" % ws if ws > 1 else "single"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "one training step = " + " + ".join(per_kernel),
                     "ms_per_kernel": per_kernel,
                     "algorithmic_bytes_per_step": bytes_step,
                     "counted_frac": None if traffic is None else traffic / (step_kernel_s * 1e9) / HBM_PEAK_GBS,
                     "per_kernel": kernel_detail,
                     "lib_sha256": library_sha256(), "counters_lib_sha256": pmc_sha,
                     "counters_match_build": pmc is not None,
                     "step_apply_fused": fused_sa,
                     "slot_scale": slot_sc,
                     "contrib_roundtrip_bytes": contrib_rt if spath != _native.PT_PATH_SAMPLED else 0,
                     "contrib_share_of_counted": None if traffic is None or spath == _native.PT_PATH_SAMPLED
                     else contrib_rt / traffic,
                     "note": "achieved / frac: SURVEY 8(d) algorithmic bytes per step over the summed kernel time "
                             "(HIP events on the launch stream). traffic / counted_bytes: (2 x FETCH_SIZE + "
                             "WRITE_SIZE) per step from rocprofv3 PMC passes (profiles/pmc_%s.json): the L2 <-> "
                             "fabric bytes, Infinity-Cache hits included (MI355X_MICROARCH.md), so it is below the "
                             "algorithmic count where repeated rows (%.1f MB entity table, hub entities, the "
                             "positive rows shared by 25 negatives) hit in L2; counted_frac = that traffic over the "
                             "same kernel time vs 8 TB/s. contrib_roundtrip_bytes: the corrupted entities' gradient "
                             "rows written by the step kernel and read back by the apply pass (fused step + apply: by each row's last "
                             "arriving wave, in the same kernel)" %
                             (args.workload, 4e-6 * dl.get_ent_tot() * dim)},
        "loss_last_step": loss_last,
    }
    if det_ms is not None:
        rec["deterministic_ms_per_step"] = det_ms
        rec["deterministic_triples_per_s"] = seq * 1e3 / det_ms
    if c3 is not None:
        rec["pu_c3"] = c3
    if c3w is not None:
        rec["pu_c3_weak"] = c3w
    if c3r is not None:
        rec["pu_c3_ref6000"] = c3r
    if c4lp is not None:
        rec["pu_c4_lp"] = c4lp
    if ws == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(path, wl, args.cpu_seconds)
    print(json.dumps(rec), flush=True)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if c4lp is not None and not c4lp["link_prediction"].get("digest_match", False):
        print("bench.py: pu_c4_lp ranks differ from the N = 1 recomputation", file=sys.stderr)
        sys.exit(4)


if __name__ == "__main__":
    main()
