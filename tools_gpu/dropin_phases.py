"""Measurement tooling: synchronized wall time of the drop-in universe leg's phases (bench.run_dropin) - each
wrapped call is bracketed by torch.cuda.synchronize(), so GPU work lands in the phase that queued it.
python tools_gpu/dropin_phases.py [c3|c4] [universes] [nosave]   (nosave: best-model checkpoints skipped, to
see the validation without the checkpoint writer's GIL share)"""
import collections
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
import torch  # noqa: E402


class A:
    pass


TIMES = collections.defaultdict(float)
COUNTS = collections.Counter()


def wrap(obj, name, label):
    f = getattr(obj, name)

    def g(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            torch.cuda.synchronize()
            TIMES[label] += time.perf_counter() - t
            COUNTS[label] += 1
    setattr(obj, name, g)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    args = A()
    args.data_dir = "/tmp/putranse_bench"
    args.universes = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    args.dim = 0
    args.valid_steps = 0
    args.link_prediction = False
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from openke.config import Parallel_Universe_Config as PUC
    mod = sys.modules[PUC.__module__]
    if "nosave" in sys.argv:
        PUC.save_model = lambda self, *a, **k: None
    bench.run_dropin(args, 1, 0, dev, name)   # warm (dataset, kernels, allocator)
    for obj, fn in ((PUC, "_train_wave"), (PUC, "_fold"), (PUC, "_ranks"), (PUC, "_checkpoint_state"),
                    (PUC, "save_parameters"), (PUC, "flush_checkpoint"), (PUC, "_materialize_maps"),
                    (PUC, "_store"), (mod, "lp_pairs_all"), (mod, "lp_pair_array"), (mod, "min_combine")):
        wrap(obj, fn, fn)
    out = bench.run_dropin(args, 1, 0, dev, name)
    print({k: v for k, v in out.items() if k != "breakdown_s"}, out["breakdown_s"])
    for k in sorted(TIMES, key=lambda k: -TIMES[k]):
        print("%-20s %3d calls %8.1f ms" % (k, COUNTS[k], TIMES[k] * 1e3))


if __name__ == "__main__":
    main()
