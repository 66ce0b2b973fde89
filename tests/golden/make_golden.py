"""Generate the golden vectors that pin the oracle and the HIP path to the reference.

Run in the build container only (the GPU box has no /root/reference):

    python tests/golden/make_golden.py

What it does
  1. ``make -C oracle ref`` compiles the reference's own C++ core from its sources where they lie
     (/root/reference/openke/base/Base.cpp) into ``oracle/_ref/Base.so`` (git-ignored).
  2. Copies the reference *Python* package to a throw-away temp dir (never into this repo), drops
     the freshly built Base.so into ``<tmp>/openke/release/`` (where its ctypes loaders look,
     TrainDataLoader.py:30-31) and imports it on CPU.
  3. Writes the synthetic datasets ``tests/golden/kg_small`` and ``kg_tiny`` (headerless format)
     and, one subprocess per case (the reference keeps process-global C state, Base.cpp:16-168),
     records inputs and outputs as compressed ``.npz`` fixtures next to this script.

The fixtures are data: inputs (seeds, configs, initial tables, batches) and the reference's
outputs (batches, losses, updated tables, universe maps, link-prediction metrics).
"""
import ctypes
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "openke-putranse_amd", "tools"))
import synth_kg  # noqa: E402

DATASETS = {"small": os.path.join(HERE, "kg_small") + os.sep, "tiny": os.path.join(HERE, "kg_tiny") + os.sep}

SAMPLER_CASES = [
    # name, dataset, threads, batch_size, neg_ent, bern, filter, seed
    ("s1", "small", 8, 375, 1, 0, 0, 7),
    ("s2", "small", 8, 123, 3, 1, 1, 11),
    ("s3", "small", 3, 50, 25, 1, 1, 4),
    ("s4", "small", 1, 64, 2, 0, 1, 0),
    ("s5", "small", 8, 5, 1, 1, 0, 3),
    ("s6", "tiny", 8, 37, 4, 1, 1, 9),
    ("s7", "tiny", 8, 16, 1, 0, 0, 2),
]

TRAIN_CASES = [
    # name, model, dim, p_norm, norm_flag, opt, lr, margin, threads, bs, neg, bern, filter, seed, torch_seed, steps
    ("t1", "TransE", 16, 1, True, "sgd", 0.5, 5.0, 8, 375, 1, 0, 0, 7, 1, 5),
    ("t2", "TransE", 32, 2, True, "sgd", 1.0, 5.0, 8, 100, 25, 1, 1, 4, 2, 3),
    ("t3", "TransE", 20, 1, True, "adagrad", 0.05, 2.0, 8, 150, 1, 0, 0, 5, 3, 6),
    ("t4", "TransH", 20, 1, True, "adagrad", 0.03, 3.0, 8, 150, 1, 0, 0, 6, 4, 5),
    ("t5", "TransH", 16, 2, True, "sgd", 0.5, 4.0, 8, 60, 4, 1, 1, 8, 5, 3),
    ("t6", "TransE", 12, 2, False, "sgd", 0.1, 3.0, 8, 200, 2, 0, 1, 9, 6, 4),
    ("t7", "TransE", 64, 2, True, "adagrad", 0.1, 1.0, 4, 90, 3, 1, 0, 10, 7, 4),
]

SAMPLER_MODE_CASES = [
    # name, dataset, threads, batch_size, neg_ent, neg_rel, bern, filter, seed, calls
    # calls: n = sampling(), h = sampling_head(), t = sampling_tail(), c = cross_sampling()
    ("m1", "small", 8, 123, 3, 0, 1, 0, 13, "hth"),
    ("m2", "small", 8, 64, 2, 2, 1, 1, 14, "nnh"),
    ("m3", "tiny", 3, 37, 1, 3, 0, 1, 15, "tccc"),
    ("m4", "small", 8, 200, 0, 1, 0, 0, 16, "nn"),
    ("m5", "small", 5, 101, 4, 1, 1, 1, 17, "cnt"),
]

UNIVERSE_CASES = [
    # name, model, dim, p_norm, n_universes, min_tc, max_tc, const_epochs, seed
    ("u1", "TransE", 8, 1, 6, 200, 400, 2, 123),
    ("u2", "TransH", 8, 1, 3, 150, 300, 2, 77),
    ("u3", "TransE", 12, 2, 4, 300, 600, 3, 5),
]

LP_CASES = [
    # name, model, dim, p_norm, torch_seed
    ("l1", "TransE", 16, 1, 21),
    ("l2", "TransH", 10, 2, 22),
]


LPT_CASES = [
    # type-constrained link prediction (Tester.run_link_prediction(type_constrain=True)); the reference
    # only reads type_constrain.txt when importTypeFiles() is called (Reader.h:352-396), so the case calls it
    # name, model, dim, p_norm, torch_seed
    ("t1", "TransE", 16, 1, 23),
    ("t2", "TransH", 10, 2, 24),
]

VAL_CASES = [
    # Validator.valid() (Validator.py:35-44): filtered hit@10 of the valid split
    # name, model, dim, p_norm, torch_seed
    ("v1", "TransE", 12, 1, 25),
    ("v2", "TransH", 8, 2, 26),
]

NBR_CASES = [
    # TrainDataLoader.get_positive_entities / get_negative_entities / get_entity_relations (Base.cpp:312-466),
    # on the full graph and after swap_helpers onto a universe
    # name, seed, universe (tc, balance) or None
    ("n1", 3, None),
    ("n2", 8, [300, 0.3]),
]

TC_CASES = [
    # name, model, dim, p_norm, torch_seed
    ("c1", "TransE", 16, 1, 31),
    ("c2", "TransH", 12, 2, 32),
]


def _import_reference(tmp):
    dst = os.path.join(tmp, "openke")
    if not os.path.exists(dst):
        shutil.copytree(os.path.join(REF, "openke"), dst)
        os.makedirs(os.path.join(dst, "release"), exist_ok=True)
        shutil.copy(os.path.join(REPO, "oracle", "_ref", "Base.so"), os.path.join(dst, "release", "Base.so"))
    sys.path.insert(0, tmp)


def _silence():
    # the reference prints from C (printf) and Python (tqdm); keep our own logs readable
    devnull = os.open(os.devnull, os.O_WRONLY)
    os.dup2(devnull, 1)


def case_glibc(out):
    libc = ctypes.CDLL("libc.so.6")
    seeds = [0, 1, 4, 5, 123, 2147483647, 4 + 17]
    vals = []
    for s in seeds:
        libc.srand(ctypes.c_uint(s))
        vals.append([libc.rand() for _ in range(400)])
    np.savez_compressed(out, seeds=np.array(seeds, dtype=np.int64), values=np.array(vals, dtype=np.int64))


def case_sampler(out, name, ds, threads, bs, neg, bern, filt, seed):
    from openke.data import TrainDataLoader
    dl = TrainDataLoader(in_path=DATASETS[ds], batch_size=bs, threads=threads, sampling_mode="normal",
                         bern_flag=bern, filter_flag=filt, neg_ent=neg, neg_rel=0, random_seed=seed)
    hs, ts, rs, ys = [], [], [], []
    for _ in range(3):
        d = dl.sampling()
        hs.append(d["batch_h"].copy()); ts.append(d["batch_t"].copy())
        rs.append(d["batch_r"].copy()); ys.append(d["batch_y"].copy())
    np.savez_compressed(out, threads=threads, batch_size=bs, neg_ent=neg, bern=bern, filter=filt, seed=seed,
                        dataset=ds, batch_h=np.stack(hs), batch_t=np.stack(ts), batch_r=np.stack(rs),
                        batch_y=np.stack(ys))


def case_sampler_mode(out, name, ds, threads, bs, neg, neg_rel, bern, filt, seed, calls):
    """sampling() with mode -1 / 1 (sampling_head / sampling_tail / cross_sampling, TrainDataLoader.py:198-246)
    and neg_rel relation corruptions (Base.cpp:233-253); the loader's full buffers are recorded."""
    from openke.data import TrainDataLoader
    dl = TrainDataLoader(in_path=DATASETS[ds], batch_size=bs, threads=threads, sampling_mode="cross",
                         bern_flag=bern, filter_flag=filt, neg_ent=neg, neg_rel=neg_rel, random_seed=seed)
    fn = {"n": dl.sampling, "h": dl.sampling_head, "t": dl.sampling_tail, "c": dl.cross_sampling}
    hs, ts, rs, ys, modes = [], [], [], [], []
    for c in calls:
        d = fn[c]()
        modes.append(d["mode"])
        hs.append(dl.batch_h.copy()); ts.append(dl.batch_t.copy())
        rs.append(dl.batch_r.copy()); ys.append(dl.batch_y.copy())
    np.savez_compressed(out, threads=threads, batch_size=bs, neg_ent=neg, neg_rel=neg_rel, bern=bern, filter=filt,
                        seed=seed, dataset=ds, calls=calls, modes=np.array(modes), batch_h=np.stack(hs),
                        batch_t=np.stack(ts), batch_r=np.stack(rs), batch_y=np.stack(ys))


def case_train(out, name, model, dim, p, norm_flag, opt, lr, margin, threads, bs, neg, bern, filt, seed, tseed,
               steps):
    import torch
    from openke.config import Trainer
    from openke.data import TrainDataLoader
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE, TransH
    from openke.module.strategy import NegativeSampling
    dl = TrainDataLoader(in_path=DATASETS["small"], batch_size=bs, threads=threads, sampling_mode="normal",
                         bern_flag=bern, filter_flag=filt, neg_ent=neg, neg_rel=0, random_seed=seed)
    torch.manual_seed(tseed)
    cls = TransE if model == "TransE" else TransH
    kge = cls(ent_tot=dl.get_ent_tot(), rel_tot=dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=norm_flag)
    init = {k: v.detach().clone().numpy() for k, v in kge.state_dict().items() if "embeddings" in k or "norm_vector" in k}
    ns = NegativeSampling(model=kge, loss=MarginLoss(margin=margin), batch_size=dl.get_batch_size())
    tr = Trainer(model=ns, data_loader=dl, train_times=0, alpha=lr, use_gpu=False, opt_method=opt)
    tr.run()  # builds the optimizer (train_times=0 runs no epoch)
    losses, bh, bt, br, snaps = [], [], [], [], []
    for s in range(steps):
        d = dl.sampling()
        bh.append(d["batch_h"].copy()); bt.append(d["batch_t"].copy()); br.append(d["batch_r"].copy())
        losses.append(tr.train_one_step(d))
        if s == 0:
            snaps.append({k: v.detach().clone().numpy() for k, v in kge.state_dict().items() if k in init})
    final = {k: v.detach().clone().numpy() for k, v in kge.state_dict().items() if k in init}
    arrs = {}
    for k in init:
        short = k.split(".")[0]
        arrs["init_" + short] = init[k]
        arrs["step1_" + short] = snaps[0][k]
        arrs["final_" + short] = final[k]
    np.savez_compressed(out, model=model, dim=dim, p_norm=p, norm_flag=norm_flag, opt=opt, lr=lr, margin=margin,
                        threads=threads, batch_size=bs, neg_ent=neg, bern=bern, filter=filt, seed=seed,
                        torch_seed=tseed, steps=steps, losses=np.array(losses, dtype=np.float64),
                        batch_h=np.stack(bh), batch_t=np.stack(bt), batch_r=np.stack(br), **arrs)


def case_universes(out, name, model, dim, p, n_univ, min_tc, max_tc, epochs, seed):
    import torch
    from openke.config import Parallel_Universe_Config
    from openke.data import TestDataLoader, TrainDataLoader
    from openke.module.model import TransE, TransH
    dl = TrainDataLoader(in_path=DATASETS["small"], nbatches=20, threads=8, sampling_mode="normal", bern_flag=0,
                         filter_flag=0, neg_ent=1, neg_rel=0, random_seed=seed)
    test_dl = TestDataLoader(dl.in_path, "link")  # re-seeds the C RNG to 4 (TestDataLoader.py:29, :88)
    cls = TransE if model == "TransE" else TransH
    pu = Parallel_Universe_Config(training_identifier=name, train_dataloader=dl, test_dataloader=test_dl,
                                  initial_num_universes=None, min_margin=1, max_margin=4, min_lr=0.001, max_lr=0.1,
                                  min_num_epochs=50, max_num_epochs=200, const_num_epochs=epochs,
                                  min_triple_constraint=min_tc, max_triple_constraint=max_tc, min_balance=0.25,
                                  max_balance=0.5, embedding_model=cls,
                                  embedding_model_param={"dim": dim, "p_norm": p, "norm_flag": 1},
                                  checkpoint_dir=tempfile.mkdtemp() + "/", valid_steps=10 ** 6, save_steps=None,
                                  training_setting="static", incremental_strategy=None)
    seed0 = pu.initial_random_seed
    # capture the per-universe draws the same way train_parallel_universes does (:320-328),
    # plus the first sampled batch of every universe (taken on a second, identical construction)
    pu.train_parallel_universes(n_univ)
    rec = {"seed0": seed0, "n_univ": n_univ}
    for u in range(n_univ):
        sp = pu.trained_embedding_spaces[u]
        ent_map = pu.entity_id_mappings[u]
        rel_map = pu.relation_id_mappings[u]
        ent_remap = np.full(len(ent_map), -1, dtype=np.int64)
        for g, l in ent_map.items():
            ent_remap[l] = g
        rel_remap = np.full(len(rel_map), -1, dtype=np.int64)
        for g, l in rel_map.items():
            rel_remap[l] = g
        rec["u%d_ent_remap" % u] = ent_remap
        rec["u%d_rel_remap" % u] = rel_remap
        rec["u%d_ent" % u] = sp.ent_embeddings.weight.detach().numpy().copy()
        rec["u%d_rel" % u] = sp.rel_embeddings.weight.detach().numpy().copy()
        if model == "TransH":
            rec["u%d_norm" % u] = sp.norm_vector.weight.detach().numpy().copy()
    # universe construction + first batch, restated from the same seeds (state after training is reset)
    for u in range(n_univ):
        pu.set_random_seed(seed0 + u)
        import random
        tc = random.randrange(min_tc, max_tc)
        bal = round(random.uniform(0.25, 0.5), 2)
        dl.compile_universe_dataset(tc, bal)
        rec["u%d_tc" % u] = tc
        rec["u%d_balance" % u] = bal
        rec["u%d_train_total" % u] = dl.lib.getTrainTotalUniverse()
        margin = random.randrange(1, 4)
        lr = round(random.uniform(0.001, 0.1), len(str(0.001).split('.')[1]))
        rec["u%d_margin" % u] = margin
        rec["u%d_lr" % u] = lr
        dl.swap_helpers()
        d = dl.sampling()
        rec["u%d_b_h" % u] = d["batch_h"].copy()
        rec["u%d_b_t" % u] = d["batch_t"].copy()
        rec["u%d_b_r" % u] = d["batch_r"].copy()
        dl.reset_universe()
    mrr_etc = pu_lp(pu)
    rec["lp"] = np.array(mrr_etc, dtype=np.float64)
    # triple classification over the universes (Parallel_Universe_Config.py:745-749 -> Tester.py:142-191)
    # from a fixed C RNG state (the negatives come from sampler thread 0)
    pu.set_random_seed(4321)
    acc, thr = pu.run_triple_classification()
    rec["tc_acc"] = float(acc)
    rec["tc_threshold"] = float(thr) if thr is not None else np.nan
    np.savez_compressed(out, model=model, dim=dim, p_norm=p, min_tc=min_tc, max_tc=max_tc, epochs=epochs, seed=seed,
                        **rec)


def pu_lp(pu):
    # Parallel_Universe_Config.run_link_prediction prints instead of returning; call the same chain
    pu.data_loader.set_sampling_mode('link')
    pu.eval_universes(eval_mode='test')
    from openke.config import Tester
    return Tester.run_link_prediction(pu, False)


def case_lp(out, name, model, dim, p, tseed):
    import torch
    from openke.config import Tester
    from openke.data import TestDataLoader
    from openke.module.model import TransE, TransH
    test_dl = TestDataLoader(DATASETS["small"], "link")
    torch.manual_seed(tseed)
    cls = TransE if model == "TransE" else TransH
    kge = cls(ent_tot=test_dl.get_ent_tot(), rel_tot=test_dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=True)
    tables = {k.split(".")[0]: v.detach().numpy().copy() for k, v in kge.state_dict().items()
              if "embeddings" in k or "norm_vector" in k}
    tester = Tester(model=kge, data_loader=test_dl, use_gpu=False)
    res = tester.run_link_prediction(type_constrain=False)
    np.savez_compressed(out, model=model, dim=dim, p_norm=p, torch_seed=tseed,
                        metrics=np.array(res, dtype=np.float64), **tables)


def write_type_file(ds_path, seed=0):
    """type_constrain.txt for a synthetic dataset (the format importTypeFiles reads, Reader.h:352-396): per
    relation the heads and tails seen with it in train/valid/test, thinned at random (so the constraint
    drops candidates that do score well) plus a few random unseen entities, and unsorted per line."""
    rng = np.random.default_rng(seed)
    trip = np.concatenate([np.loadtxt(ds_path + f, dtype=np.int64, ndmin=2)
                           for f in ("train2id.txt", "valid2id.txt", "test2id.txt")])
    with open(ds_path + "entity2id.txt") as f:
        E = sum(1 for _ in f)
    with open(ds_path + "relation2id.txt") as f:
        R = sum(1 for _ in f)
    lines = [str(R)]
    for r in range(R):
        sel = trip[trip[:, 2] == r]
        for col in (0, 1):
            ents = np.unique(sel[:, col])
            keep = ents[rng.random(len(ents)) < 0.7]
            extra = rng.integers(0, E, size=int(rng.integers(0, 6)))
            vals = np.unique(np.concatenate([keep, extra]))
            rng.shuffle(vals)
            lines.append(" ".join([str(r), str(len(vals))] + [str(int(v)) for v in vals]))
    with open(ds_path + "type_constrain.txt", "w") as f:
        f.write("\n".join(lines) + "\n")


def case_lpt(out, name, model, dim, p, tseed):
    import torch
    from openke.config import Tester
    from openke.data import TestDataLoader
    from openke.module.model import TransE, TransH
    test_dl = TestDataLoader(DATASETS["small"], "link")
    test_dl.lib.importTypeFiles()
    torch.manual_seed(tseed)
    cls = TransE if model == "TransE" else TransH
    kge = cls(ent_tot=test_dl.get_ent_tot(), rel_tot=test_dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=True)
    tables = {k.split(".")[0]: v.detach().numpy().copy() for k, v in kge.state_dict().items()
              if "embeddings" in k or "norm_vector" in k}
    tester = Tester(model=kge, data_loader=test_dl, use_gpu=False)
    res = tester.run_link_prediction(type_constrain=True)
    plain = [tester.lib.getTestLinkMRR(0), tester.lib.getTestLinkMR(0), tester.lib.getTestLinkHit10(0),
             tester.lib.getTestLinkHit3(0), tester.lib.getTestLinkHit1(0)]
    np.savez_compressed(out, model=model, dim=dim, p_norm=p, torch_seed=tseed,
                        metrics_tc=np.array(res, dtype=np.float64), metrics=np.array(plain, dtype=np.float64),
                        **tables)


def case_val(out, name, model, dim, p, tseed):
    import torch
    from openke.config import Validator
    from openke.data import TestDataLoader
    from openke.module.model import TransE, TransH
    valid_dl = TestDataLoader(DATASETS["small"], "link", mode='valid')
    torch.manual_seed(tseed)
    cls = TransE if model == "TransE" else TransH
    kge = cls(ent_tot=valid_dl.get_ent_tot(), rel_tot=valid_dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=True)
    tables = {k.split(".")[0]: v.detach().numpy().copy() for k, v in kge.state_dict().items()
              if "embeddings" in k or "norm_vector" in k}
    validator = Validator(model=kge, data_loader=valid_dl)
    hit10 = validator.valid()
    np.savez_compressed(out, model=model, dim=dim, p_norm=p, torch_seed=tseed, hit10=float(hit10), **tables)


def case_nbr(out, name, seed, uni):
    from openke.data import TrainDataLoader
    dl = TrainDataLoader(in_path=DATASETS["small"], batch_size=50, threads=8, sampling_mode="normal", bern_flag=0,
                         filter_flag=0, neg_ent=1, neg_rel=0, random_seed=seed)
    if uni is not None:
        dl.compile_universe_dataset(uni[0], uni[1])
        dl.swap_helpers()
    E, R = dl.lib.getEntityTotal(), dl.lib.getRelationTotal()
    rng = np.random.default_rng(seed)
    queries = [(int(rng.integers(0, E)), int(rng.integers(0, R)), int(rng.integers(0, 2))) for _ in range(40)]
    rec = {"queries": np.array(queries, dtype=np.int64), "ent_total": E, "rel_total": R}
    for i, (e, r, f) in enumerate(queries):
        rec["pos_%d" % i] = dl.get_positive_entities(e, r, f)
        rec["neg_%d" % i] = dl.get_negative_entities(e, r, f)
        rec["rels_%d" % i] = dl.get_entity_relations(e, f)
    np.savez_compressed(out, seed=seed, universe=np.array(uni if uni is not None else [], dtype=np.float64), **rec)


def case_tc(out, name, model, dim, p, tseed):
    """Tester.run_triple_classification on a random-init model (Tester.py:142-191), then one more
    getTestBatch call of the same loader (the negatives continue the thread-0 stream)."""
    import torch
    from openke.config import Tester
    from openke.data import TestDataLoader
    from openke.module.model import TransE, TransH
    test_dl = TestDataLoader(DATASETS["small"], "classification")
    torch.manual_seed(tseed)
    cls = TransE if model == "TransE" else TransH
    kge = cls(ent_tot=test_dl.get_ent_tot(), rel_tot=test_dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=True)
    tables = {k.split(".")[0]: v.detach().numpy().copy() for k, v in kge.state_dict().items()
              if "embeddings" in k or "norm_vector" in k}
    tester = Tester(model=kge, data_loader=test_dl, use_gpu=False)
    acc, thr = tester.run_triple_classification()
    pos, neg = next(iter(test_dl))
    np.savez_compressed(out, model=model, dim=dim, p_norm=p, torch_seed=tseed, acc=float(acc), threshold=float(thr),
                        pos_h=pos["batch_h"].copy(), pos_t=pos["batch_t"].copy(), pos_r=pos["batch_r"].copy(),
                        neg_h=neg["batch_h"].copy(), neg_t=neg["batch_t"].copy(), neg_r=neg["batch_r"].copy(),
                        **tables)


# ------------------------------------------------------------------------------------------------------------------
# Real scale (round 6): the reference's own benchmark data and trained tables (SURVEY §8c fixture recipe).
# The folders are packed into tests/golden/real_<name>.npz (realdata.pack_dataset) and the reference is run on the
# folder realdata.write_dataset rebuilds from them, i.e. on exactly what the tests read.
#   wn18:  benchmarks/WN18 as it is (train / valid / test, type_constrain.txt), E = 40,943, R = 18.
#   fb15k: benchmarks/FB15K has no train2id.txt (.MISSING_LARGE_BLOBS:1), so the folder takes its valid split
#          (50,000 triples) as train2id.txt, test2id.txt lines 300-599 as valid2id.txt and lines 0-299 as
#          test2id.txt; E = 14,951, R = 1,345.
# Checkpoints are read with torch.load(weights_only=True) only.
REAL_DATA = {"wn18": os.path.join(HERE, "real_wn18.npz"), "fb15k": os.path.join(HERE, "real_fb15k.npz")}

REAL_LP_CASES = [
    # name, dataset, checkpoint (best_models/), model, p_norm, type_constrain, queries whose score vectors are kept
    ("wn18h", "wn18", "transH_WN18_optimal_model.ckpt", "TransH", 1, True, [0]),
    ("fb15ke", "fb15k", "transe_FB15K_optimal_model.ckpt", "TransE", 2, False, [0, 150]),
]

REAL_SAMPLER_CASES = [
    # name, batch_size, neg_ent, bern, filter, seed, calls (WN18, 8 threads); C1's bs 1414 and 100, and C2's
    # bs 2000 x 25 negatives on WN18's graph
    ("w1", 1414, 1, 0, 0, 4, 6),
    ("w2", 1414, 1, 1, 1, 4, 6),
    ("w3", 100, 1, 0, 1, 7, 6),
    ("w4", 100, 1, 1, 0, 7, 6),
    ("w5", 2000, 25, 1, 1, 4, 4),
]


def _sha1(*arrays):
    import hashlib
    m = hashlib.sha1()
    for a in arrays:
        m.update(np.ascontiguousarray(a, dtype=np.int64).tobytes())
    return m.hexdigest()


def _real_dir(tmp, name):
    sys.path.insert(0, os.path.dirname(HERE))
    import realdata
    return realdata.write_dataset(REAL_DATA[name], os.path.join(tmp, "real_" + name))


def case_real_lp(out, name, ds, ckpt, model, p, tc, vec_queries):
    """Tester.run_link_prediction (Tester.py:70-93) on a reference-trained table over the full entity set, plus
    every query's raw / filtered (and type-constrained) counts as testHead / testTail compute them
    (Test.h:118-359): the loop of run_link_prediction, with the accumulators zeroed before each query and read
    after it (they are exact integers there)."""
    import torch
    from openke.config import Tester
    from openke.data import TestDataLoader
    from openke.module.model import TransE, TransH
    path = _real_dir(TMP, ds)
    test_dl = TestDataLoader(path, "link")
    if tc:
        test_dl.lib.importTypeFiles()   # the reference's Python never calls it
    sd = torch.load(os.path.join(REF, "best_models", ckpt), weights_only=True, map_location="cpu")
    dim = sd["ent_embeddings.weight"].shape[1]
    cls = TransE if model == "TransE" else TransH
    kge = cls(ent_tot=test_dl.get_ent_tot(), rel_tot=test_dl.get_rel_tot(), dim=dim, p_norm=p, norm_flag=True)
    kge.load_state_dict(sd)
    tables = {k.split(".")[0]: v.detach().numpy().copy() for k, v in kge.state_dict().items()
              if "embeddings" in k or "norm_vector" in k}
    tester = Tester(model=kge, data_loader=test_dl, use_gpu=False)
    res = tester.run_link_prediction(type_constrain=bool(tc))
    lib = tester.lib
    plain = [lib.getTestLinkMRR(0), lib.getTestLinkMR(0), lib.getTestLinkHit10(0), lib.getTestLinkHit3(0),
             lib.getTestLinkHit1(0)]
    names = ["l_rank", "l_filter_rank", "r_rank", "r_filter_rank"]
    if tc:
        names += [n + "_constrain" for n in names]
    acc = [ctypes.c_float.in_dll(lib, n) for n in names]
    test_dl.set_sampling_mode("link")
    n = lib.getTestTotal()
    ranks = np.zeros((len(names), n), dtype=np.int32)
    queries = np.zeros((n, 3), dtype=np.int32)
    vecs_h, vecs_t = [], []
    for index, (dh, dt) in enumerate(test_dl):
        for a in acc:
            a.value = 0.0
        sh = tester.test_one_step(dh)
        lib.testHead(sh.__array_interface__["data"][0], index, int(tc))
        st = tester.test_one_step(dt)
        lib.testTail(st.__array_interface__["data"][0], index, int(tc))
        ranks[:, index] = [int(a.value) - 1 for a in acc]   # accumulated 1 + count
        queries[index] = (dh["batch_h"][0], dh["batch_t"][0], dh["batch_r"][0])
        if index in vec_queries:
            vecs_h.append(np.asarray(sh, dtype=np.float32).copy())
            vecs_t.append(np.asarray(st, dtype=np.float32).copy())
    np.savez_compressed(out, dataset=ds, checkpoint=ckpt, model=model, dim=dim, p_norm=p, type_constrain=int(tc),
                        metrics=np.array(plain, dtype=np.float64),
                        metrics_tc=np.array(res if tc else plain, dtype=np.float64),
                        rank_names=np.array(names), ranks=ranks, queries=queries,
                        vec_queries=np.array(vec_queries, dtype=np.int64), vec_head=np.stack(vecs_h),
                        vec_tail=np.stack(vecs_t), **tables)


def case_real_sampler(out, bs, neg, bern, filt, seed, calls):
    """sampling() (Base.cpp:266-310) on WN18: SHA-1 of each call's (h, t, r) int64 arrays, the first call kept."""
    from openke.data import TrainDataLoader
    path = _real_dir(TMP, "wn18")
    dl = TrainDataLoader(in_path=path, batch_size=bs, threads=8, sampling_mode="normal", bern_flag=bern,
                         filter_flag=filt, neg_ent=neg, neg_rel=0, random_seed=seed)
    digests, first = [], None
    for c in range(calls):
        d = dl.sampling()
        digests.append(_sha1(d["batch_h"], d["batch_t"], d["batch_r"]))
        if c == 0:
            first = np.stack([d["batch_h"], d["batch_t"], d["batch_r"]]).astype(np.int32)
    np.savez_compressed(out, batch_size=bs, neg_ent=neg, bern=bern, filter=filt, seed=seed, calls=calls,
                        digests=np.array(digests), first=first)


def case_real_universes(out, seeds, tc_range, bal_range):
    """The per-universe protocol on WN18 (Parallel_Universe_Config.py:157-161, 209-226; UniverseConstructor.h:
    327-397): set_random_seed(s), randrange(tc), uniform(balance), getParallelUniverse; remaps, universe sizes,
    then swapHelpers and two sampling() calls of the universe (nbatches 20) as SHA-1 digests."""
    import random
    from openke.data import TrainDataLoader
    path = _real_dir(TMP, "wn18")
    dl = TrainDataLoader(in_path=path, nbatches=20, threads=8, sampling_mode="normal", bern_flag=0, filter_flag=0,
                         neg_ent=1, neg_rel=0, random_seed=4)
    rec = {"seeds": np.array(seeds, dtype=np.int64)}
    for s in seeds:
        dl.lib.setRandomSeed(s)
        dl.lib.randReset()
        random.seed(s)
        tc = random.randrange(*tc_range)
        bal = round(random.uniform(*bal_range), 2)
        dl.compile_universe_dataset(tc, bal)
        em, rm = dl.get_universe_mappings()
        rec["s%d_tc" % s], rec["s%d_balance" % s] = tc, bal
        rec["s%d_train_total" % s] = dl.lib.getTrainTotalUniverse()
        rec["s%d_batch_size" % s] = dl.batch_size
        rec["s%d_ent_remap" % s] = em.astype(np.int32)
        rec["s%d_rel_remap" % s] = rm.astype(np.int32)
        dl.swap_helpers()
        digests = []
        for _ in range(2):   # (sampling() returns the same buffers each call: hash each batch before the next)
            d = dl.sampling()
            digests.append(_sha1(d["batch_h"], d["batch_t"], d["batch_r"]))
        rec["s%d_digests" % s] = np.array(digests)
        dl.reset_universe()
    np.savez_compressed(out, tc_range=np.array(tc_range), bal_range=np.array(bal_range), **rec)


def pack_real_data():
    sys.path.insert(0, os.path.dirname(HERE))
    import realdata
    bench = os.path.join(REF, "benchmarks")
    if not os.path.exists(REAL_DATA["wn18"]):
        src = os.path.join(bench, "WN18")
        realdata.pack_dataset(REAL_DATA["wn18"], 40943, 18,
                              {f: realdata.read_triples(os.path.join(src, f)) for f in realdata.SPLITS},
                              type_file=os.path.join(src, "type_constrain.txt"),
                              source="benchmarks/WN18/{train,valid,test}2id.txt, type_constrain.txt")
    if not os.path.exists(REAL_DATA["fb15k"]):
        src = os.path.join(bench, "FB15K")
        test = realdata.read_triples(os.path.join(src, "test2id.txt"))
        realdata.pack_dataset(REAL_DATA["fb15k"], 14951, 1345,
                              {"train2id.txt": realdata.read_triples(os.path.join(src, "valid2id.txt")),
                               "valid2id.txt": test[300:600], "test2id.txt": test[:300]},
                              source="benchmarks/FB15K: train2id := valid2id.txt (train2id.txt is not in the "
                                     "reference), valid2id := test2id.txt[300:600], test2id := test2id.txt[:300]")


TMP = None


def run_case(kind, args_json, out, tmp):
    global TMP
    TMP = tmp
    args = json.loads(args_json)
    _import_reference(tmp)
    _silence()
    {"glibc": case_glibc, "sampler": case_sampler, "sampler_mode": case_sampler_mode, "train": case_train, "universes": case_universes,
     "lp": case_lp, "lpt": case_lpt, "val": case_val, "nbr": case_nbr, "tc": case_tc, "real_lp": case_real_lp,
     "real_sampler": case_real_sampler, "real_universes": case_real_universes}[kind](out, *args)


def main():
    subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "ref"])
    for ds, path in DATASETS.items():
        if not os.path.exists(os.path.join(path, "test2id.txt")):
            synth_kg.write_dataset(path, *synth_kg.SHAPES[ds], seed=0, ent_skew=synth_kg.ENT_SKEW[ds])
    if not os.path.exists(DATASETS["small"] + "type_constrain.txt"):
        write_type_file(DATASETS["small"])
    tmp = tempfile.mkdtemp(prefix="refpy_")
    jobs = [("glibc", [], "glibc_rand.npz")]
    jobs += [("sampler", list(c), "sampler_%s.npz" % c[0]) for c in SAMPLER_CASES]
    jobs += [("sampler_mode", list(c), "samplermode_%s.npz" % c[0]) for c in SAMPLER_MODE_CASES]
    jobs += [("train", list(c), "train_%s.npz" % c[0]) for c in TRAIN_CASES]
    jobs += [("universes", list(c), "universes_%s.npz" % c[0]) for c in UNIVERSE_CASES]
    jobs += [("lp", list(c), "lp_%s.npz" % c[0]) for c in LP_CASES]
    jobs += [("lpt", list(c), "lpt_%s.npz" % c[0]) for c in LPT_CASES]
    jobs += [("val", list(c), "val_%s.npz" % c[0]) for c in VAL_CASES]
    jobs += [("nbr", list(c), "nbr_%s.npz" % c[0]) for c in NBR_CASES]
    jobs += [("tc", list(c), "tc_%s.npz" % c[0]) for c in TC_CASES]
    pack_real_data()
    jobs += [("real_lp", list(c), "reallp_%s.npz" % c[0]) for c in REAL_LP_CASES]
    jobs += [("real_sampler", list(c[1:]), "realsampler_%s.npz" % c[0]) for c in REAL_SAMPLER_CASES]
    jobs += [("real_universes", [list(range(4, 12)), [500, 2000], [0.25, 0.5]], "realuniverses_wn18.npz")]
    only = sys.argv[1:]
    for kind, args, fname in jobs:
        if only and not any(fname.startswith(o) for o in only):
            continue
        out = os.path.join(HERE, fname)
        print("generating", fname, flush=True)
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--case", kind, json.dumps(args), out, tmp])
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--case":
        run_case(*sys.argv[2:6])
    else:
        main()
