"""One rank of the end-to-end multi-rank PuTransE flow (tests/test_gpu_pu.py::test_multi_rank_pu_flow_matches_
single_process), run as a fresh process: Parallel_Universe_Config(deterministic=True) over gloo with every rank
on cuda:0 - train_parallel_universes (training waves placed by LPT, validation and early-stopping bookkeeping,
best-model checkpoints), save_model, load_parameters into a fresh config, run_link_prediction.

  python tests/dist_pu_worker.py RANK WORLD PORT OUT_DIR

Rank 0 writes OUT_DIR/result_w<WORLD>.json (validation schedule, final bookkeeping, metrics, ranks) next to the
checkpoints under OUT_DIR/ckpt_w<WORLD>/."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "openke-putranse_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

KG_SMALL = os.path.join(HERE, "golden", "kg_small") + os.sep
N_UNIVERSES, VALID_STEPS, WAVE = 12, 4, 6


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    import torch.distributed as dist
    torch.cuda.set_device(0)
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = port
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from openke.config import Parallel_Universe_Config
    from openke.data import TestDataLoader, TrainDataLoader
    from openke.module.model import TransE

    def config(ck):
        dl = TrainDataLoader(in_path=KG_SMALL, nbatches=20, threads=8, sampling_mode="normal", bern_flag=0,
                             filter_flag=0, neg_ent=1, neg_rel=0, random_seed=4)
        test_dl = TestDataLoader(dl.in_path, "link")
        return Parallel_Universe_Config(
            training_identifier="dist", train_dataloader=dl, test_dataloader=test_dl, initial_num_universes=None,
            min_margin=1, max_margin=4, min_lr=0.001, max_lr=0.1, const_num_epochs=3, min_triple_constraint=150,
            max_triple_constraint=400, min_balance=0.25, max_balance=0.5, embedding_model=TransE,
            embedding_model_param={"dim": (8, 24), "p_norm": 1, "norm_flag": 1}, checkpoint_dir=ck,
            valid_steps=VALID_STEPS, early_stopping_patience=100, save_steps=6, training_setting="static",
            incremental_strategy=None, universe_wave_size=WAVE, deterministic=True)

    ck = os.path.join(out, "ckpt_w%d" % world) + os.sep
    os.makedirs(ck, exist_ok=True)
    cfg = config(ck)
    schedule = []
    valid = cfg.valid

    def logged_valid():
        h = valid()
        schedule.append(h)
        return h
    cfg.valid = logged_valid
    cfg.train_parallel_universes(N_UNIVERSES)
    owners = {int(u): int(r) for u, r in cfg.universe_owners.items()}
    cfg.save_model("final.ckpt")
    re = config(ck)
    re.load_parameters("final.ckpt")
    met = re.run_link_prediction()
    if rank == 0:
        with open(os.path.join(out, "result_w%d.json" % world), "w") as f:
            json.dump({"schedule": schedule, "best_hit10": cfg.best_hit10, "bad_counts": cfg.bad_counts,
                       "next_universe_id": cfg.next_universe_id, "metrics": [float(x) for x in met],
                       "ranks": [np.asarray(x).tolist() for x in re.last_ranks], "owners": owners,
                       "ranks_per_universe": sorted(set(owners.values()))}, f)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
