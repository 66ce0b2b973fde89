"""The universe trainer's concurrent class launches overlap whatever streams the calling process already holds.

A set whose universes fall into several shape classes runs one persistent launch per class, side by side, each
over its share of the CUs (pt_universe_set_create). Round 4 launched them on the caller's stream plus per-set side
streams: in a process that already held streams (torch's, the C2 trainer's capture stream) two class launches
shared one of the process's GPU_MAX_HW_QUEUES hardware queues and ran one after the other (the driver's default
bench line: C3 58.7 ms against 35.7 ms standalone). The launches now run on process-wide streams with hardware
queues of their own (class_streams, capi.cpp). This test holds a stream of its own, trains a four-launch set and
checks from pt_universe_set_launch_times that every launch started before any other finished. The trained tables
are checked elsewhere (test_gpu_pu.py, test_gpu_configs.py); here only the schedule."""
import ctypes

import numpy as np
import pytest
import torch

from conftest import KG_SMALL

pytestmark = pytest.mark.gpu


def _job(L, _native, h, dim, epochs, dev, keep):
    E, R, N = L.pt_universe_ent_total(h), L.pt_universe_rel_total(h), L.pt_universe_train_total(h)
    g = torch.Generator().manual_seed(dim)
    ent = ((torch.rand(E, dim, generator=g) - 0.5) * 0.2).to(dev)
    rel = ((torch.rand(R, dim, generator=g) - 0.5) * 0.2).to(dev)
    accs = (torch.zeros_like(ent), torch.zeros_like(rel))
    st = np.zeros(8, dtype=np.uint64)
    _native.check(L.pt_universe_seeds(h, st.ctypes.data))
    keep.append((ent, rel, accs, st))
    j = _native.UniverseJob()
    j.graph = L.pt_universe_graph(h)
    j.seeds = st.ctypes.data
    j.threads, j.batch_size, j.epochs, j.nbatches, j.neg = 8, max(N // 20, 1), epochs, 20, 1
    j.lr, j.margin = 0.05, 2.0
    j.ent, j.rel, j.normv = ent.data_ptr(), rel.data_ptr(), None
    j.ent_acc, j.rel_acc, j.norm_acc = accs[0].data_ptr(), accs[1].data_ptr(), None
    j.dim = dim
    return j


def test_class_launches_overlap_beside_other_streams():
    from openke import _native
    L = _native.lib()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    # the process already holds a stream of its own beside torch's (as the default bench process holds the C2
    # trainer's capture stream when it trains the C3 set), used once so its hardware queue is taken
    hip = ctypes.CDLL("libamdhip64.so")
    extra = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(extra), 1) == 0
    scratch = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    assert hip.hipMemsetAsync(ctypes.c_void_p(scratch.data_ptr()), 0, ctypes.c_size_t(1 << 20), extra) == 0
    assert hip.hipStreamSynchronize(extra) == 0
    torch.ones(1024, device=dev).sum().item()
    g = ctypes.c_void_p()
    _native.check(L.pt_graph_load(KG_SMALL.encode(), ctypes.byref(g)))
    # dims of four row-shape launches: a class-0 shape and three class-1 shapes (the longest become hot kernels)
    dims = [8, 69, 61, 23, 8, 69, 61, 23]
    n = len(dims)
    seeds = np.array([100 + k for k in range(n)], dtype=np.int64)
    tcs = np.full(n, 1500, dtype=np.int64)
    bals = np.full(n, 0.3, dtype=np.float32)
    handles = (ctypes.c_void_p * n)()
    _native.check(L.pt_universe_build_many(g, n, seeds.ctypes.data, 8, tcs.ctypes.data, bals.ctypes.data, 0,
                                           handles))
    keep = []
    try:
        jobs = [_job(L, _native, handles[i], dims[i], 40, dev, keep) for i in range(n)]
        arr = (_native.UniverseJob * n)(*jobs)
        us = ctypes.c_void_p()
        _native.check(L.pt_universe_set_create(arr, n, 0, 1, 1, _native.PT_ADAGRAD, 0, 0, ctypes.byref(us)))
        try:
            losses = torch.zeros(sum(int(j.epochs) for j in jobs), device=dev)
            _native.check(L.pt_universe_set_train(us, _native.ptr(losses), _native.stream()))
            torch.cuda.synchronize()
            assert torch.isfinite(losses).all()
            cnt = ctypes.c_int64(0)
            _native.check(L.pt_universe_set_launch_times(us, 0, None, ctypes.byref(cnt)))
            assert cnt.value >= 3, "the set should take several class launches, got %d" % cnt.value
            buf = np.zeros(3 * cnt.value, dtype=np.float32)
            _native.check(L.pt_universe_set_launch_times(us, cnt.value, buf.ctypes.data, ctypes.byref(cnt)))
            rows = buf.reshape(-1, 3)
            starts, ends = rows[:, 0], rows[:, 1]
            assert int(rows[:, 2].sum()) == n
            # concurrent: every launch started before the first one ended (one queue per launch)
            assert starts.max() < 0.5 * ends.min(), rows.tolist()
        finally:
            L.pt_universe_set_free(us)
    finally:
        for i in range(n):
            L.pt_universe_free(handles[i])
        L.pt_graph_free(g)
        hip.hipStreamDestroy(extra)
