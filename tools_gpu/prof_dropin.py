"""Measurement tooling: cProfile of the drop-in universe leg (bench.run_dropin) - where the host time of
Parallel_Universe_Config.train_parallel_universes goes.  python tools_gpu/prof_dropin.py [c3|c4] [universes]"""
import cProfile
import os
import pstats
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
import torch  # noqa: E402


class A:
    pass


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
    bench.run_dropin(args, 1, 0, dev, name)   # warm (dataset, kernels, allocator)
    pr = cProfile.Profile()
    pr.enable()
    out = bench.run_dropin(args, 1, 0, dev, name)
    pr.disable()
    print({k: v for k, v in out.items() if k != "breakdown_s"}, out["breakdown_s"])
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(45)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
