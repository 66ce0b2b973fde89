"""Diagnostic (measurement tooling, not product code): one C2-shaped training step through the fused step + apply
kernel and through the step + apply pair from the same tables and sampler streams; reports the entity / relation
rows that differ, classified by how the step touched them (a positive's h / t, a corrupted entity's bucket), and
whether two fused runs agree with each other.

  python tools_gpu/diag_sa.py [--steps N] [--bs B] [--neg K]
"""
import argparse
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "openke-putranse_amd"))
sys.path.insert(0, os.path.join(REPO, "openke-putranse_amd", "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--bs", type=int, default=2000)
    ap.add_argument("--neg", type=int, default=25)
    ap.add_argument("--dim", type=int, default=200)
    args = ap.parse_args()
    import synth_kg
    from openke import _native
    from openke.config import Trainer
    from openke.data import TrainDataLoader
    from openke.module.loss import MarginLoss
    from openke.module.model import TransE
    from openke.module.strategy import NegativeSampling
    path = synth_kg.ensure_dataset(os.path.join(tempfile.gettempdir(), "putranse_bench"), "fb15k237")
    bs, neg = args.bs, args.neg

    def loader():
        return TrainDataLoader(in_path=path, batch_size=bs, threads=8, sampling_mode="normal", bern_flag=1,
                               filter_flag=1, neg_ent=neg, neg_rel=0, random_seed=4)

    d = loader().sampling()
    h, t = d["batch_h"], d["batch_t"]
    pos_rows = set(h[:bs].tolist()) | set(t[:bs].tolist())
    corrupted = np.where(h[bs:] != np.tile(h[:bs], neg), h[bs:], t[bs:])
    bucket = np.bincount(corrupted, minlength=20000)

    def run(fused):
        dl = loader()
        dl.nbatches = args.steps
        torch.manual_seed(0)
        kge = TransE(dl.get_ent_tot(), dl.get_rel_tot(), dim=args.dim, p_norm=2, norm_flag=True)
        ns = NegativeSampling(model=kge, loss=MarginLoss(margin=5.0), batch_size=bs)
        tr = Trainer(model=ns, data_loader=dl, train_times=1, alpha=1.0, use_gpu=True)
        tr._setup()
        _native.check(_native.lib().pt_trainer_set_step_apply(tr._native, fused))
        tr.run()
        torch.cuda.synchronize()
        assert _native.lib().pt_trainer_step_apply(tr._native) == fused
        return (tr.last_epoch_loss, kge.ent_embeddings.weight.detach().cpu().numpy().copy(),
                kge.rel_embeddings.weight.detach().cpu().numpy().copy())

    pair = run(0)
    f1 = run(1)
    f2 = run(1)
    print("loss pair %.7f fused %.7f %.7f" % (pair[0], f1[0], f2[0]))
    for name, f in (("fused1", f1), ("fused2", f2)):
        de = np.abs(f[1] - pair[1]).max(axis=1)
        dr = np.abs(f[2] - pair[2]).max(axis=1)
        bad = np.nonzero(de > 1e-6)[0]
        print("%s: ent rows off %d (max %.3g), rel rows off %d (max %.3g)" % (name, len(bad), de.max(), int((dr > 1e-6).sum()),
                                                                            dr.max()))
        if len(bad):
            inpos = np.array([b in pos_rows for b in bad])
            bk = bucket[bad]
            print("   of them: positive h/t %d, bucket>0 %d, both %d, neither %d; bucket sizes %s" %
                  (inpos.sum(), (bk > 0).sum(), (inpos & (bk > 0)).sum(), (~inpos & (bk == 0)).sum(),
                   np.bincount(bk)[:12].tolist()))
            print("   first rows", bad[:10].tolist(), "errs", np.round(de[bad[:10]], 7).tolist())
    d12 = np.abs(f1[1] - f2[1]).max(axis=1)
    print("fused1 vs fused2: ent rows off %d (max %.3g)" % (int((d12 > 1e-6).sum()), d12.max()))
    touched = pos_rows | set(np.nonzero(bucket)[0].tolist())
    print("rows touched by the step: %d (positive h/t %d)" % (len(touched), len(pos_rows)))


if __name__ == "__main__":
    main()
