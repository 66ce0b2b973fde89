# coding:utf-8
"""Trainer (mirror of openke/config/Trainer.py:12-138).

Same constructor, attributes and setters. run() keeps the epoch/batch loop of Trainer.py:91-100 but
each epoch is ONE replayed hipGraph of `nbatches` fused steps: every step samples its batch inside the
kernel from the data loader's stream (bit-identical to TrainDataLoader.sampling()), computes
NegativeSampling + MarginLoss forward and the analytic backward, and applies SGD or Adagrad to the
touched rows only (identical to the reference's dense update). Losses stay on the device until the
end of the epoch (one host sync per epoch instead of one per step). Cross sampling and relation
corruption (neg_rel > 0) train batch by batch: GPU-sampled batch, then the external-batch step."""
import ctypes
import os

import numpy as np
import torch
from tqdm import tqdm

from .. import _native
from ..module.loss import MarginLoss
from ..module.model.Model import Model
from ..module.strategy import NegativeSampling


class NativeOptimizer(object):
    """Optimizer state of the fused path (Adagrad state_sum per table, eps 1e-10, lr_decay 0,
    initial accumulator 0 — torch.optim.Adagrad defaults used by Trainer.py:64-70)."""

    def __init__(self, method, lr, tables):
        self.method = method
        self.lr = lr
        self.state_sum = tuple(torch.zeros_like(t) if (t is not None and method == _native.PT_ADAGRAD) else None
                               for t in tables)

    def zero_grad(self):
        pass


class Trainer(object):

    def __init__(self, model=None, data_loader=None, valid_dataloader=None, train_times=1000, alpha=0.5,
                 use_gpu=True, opt_method="sgd", save_steps=None, checkpoint_dir=None, deterministic=False):
        self.work_threads = 8
        self.train_times = train_times
        self.opt_method = opt_method
        self.optimizer = None
        self.lr_decay = 0
        self.weight_decay = 0
        self.alpha = alpha
        self.model = model
        self.data_loader = data_loader
        self.use_gpu = use_gpu
        self.save_steps = save_steps
        self.checkpoint_dir = checkpoint_dir
        self._native = None
        self._native_key = None
        # reference-order mode (pt_trainer_set_deterministic): per-row gradient sums in slot order, lookup by
        # lookup, as embedding_dense_backward does (bit-identical run to run); off = the fused fast path
        self.deterministic = bool(deterministic)

    # ------------------------------------------------------------------ native setup ------------
    def _parts(self):
        ns = self.model
        if not isinstance(ns, NegativeSampling):
            raise NotImplementedError("the accelerated Trainer trains NegativeSampling(TransE|TransH, MarginLoss)")
        kge, loss = ns.model, ns.loss
        if not isinstance(kge, Model) or kge.native_model is None:
            raise NotImplementedError("model %s is outside the accelerated path" % type(kge).__name__)
        if not isinstance(loss, MarginLoss) or loss.adv_flag:
            raise NotImplementedError("only MarginLoss without adversarial temperature is accelerated")
        if ns.regul_rate != 0 or ns.l3_regul_rate != 0:
            raise NotImplementedError("regularisation is outside the accelerated path")
        if self.lr_decay != 0 or self.weight_decay != 0:
            raise NotImplementedError("lr_decay / weight_decay are 0 in the reference path")
        return ns, kge, loss

    def _setup(self):
        _native.require_gpu()
        ns, kge, loss = self._parts()
        ns.cuda()
        if self.optimizer is None:
            m = self.opt_method
            if m in ("Adagrad", "adagrad"):
                method = _native.PT_ADAGRAD
            elif m in ("Adadelta", "adadelta", "Adam", "adam"):
                raise NotImplementedError("%s is outside the accelerated path (SGD and Adagrad are)" % m)
            else:
                method = _native.PT_SGD
            self.optimizer = NativeOptimizer(method, self.alpha, kge.tables())
        opt = self.optimizer
        margin = float(loss.margin.item())
        desc = kge.native_desc(opt.method, opt.lr, margin, opt.state_sum)
        key = (id(kge), kge.tables()[0].data_ptr(), opt.method, opt.lr, margin)
        L = _native.lib()
        if self._native is None:
            h = ctypes.c_void_p()
            _native.check(L.pt_trainer_create(ctypes.byref(desc), ctypes.byref(h)))
            self._native = h
        elif key != self._native_key:
            _native.check(L.pt_trainer_update_desc(self._native, ctypes.byref(desc)))
        self._native_key = key
        _native.check(L.pt_trainer_set_deterministic(self._native, 1 if self.deterministic else 0))
        return ns, kge, loss

    def __del__(self):
        if getattr(self, "_native", None) is not None:
            try:
                torch.cuda.synchronize()
                _native.lib().pt_trainer_free(self._native)
            except Exception:
                pass
            self._native = None

    # ------------------------------------------------------------------ reference API -----------
    def train_one_step(self, data):
        """One step on an explicitly given batch (Trainer.py:44-56); returns loss.item()."""
        ns, kge, loss = self._setup()
        dev = kge.ent_embeddings.weight.device
        bs = ns.batch_size
        h = torch.as_tensor(np.asarray(data['batch_h']), dtype=torch.int64).to(dev).contiguous()
        t = torch.as_tensor(np.asarray(data['batch_t']), dtype=torch.int64).to(dev).contiguous()
        r = torch.as_tensor(np.asarray(data['batch_r']), dtype=torch.int64).to(dev).contiguous()
        mode = data.get('mode', 'normal')
        if mode != 'normal':
            # head_batch / tail_batch (TransE.py:51-58, TransH.py:66-73): the uncorrupted side and the
            # relation are given once per positive and broadcast over the negatives - the same slots as
            # the expanded normal-mode batch (the score adds h + (r - t) instead of (h + r) - t there:
            # fp32 association only)
            if mode not in ('head_batch', 'tail_batch'):
                raise ValueError("unknown batch mode %r" % (mode,))
            full = h if mode == 'head_batch' else t
            rep = full.numel() // max(bs, 1)
            if mode == 'head_batch':
                t = t[:bs].repeat(rep)
            else:
                h = h[:bs].repeat(rep)
            r = r[:bs].repeat(rep)
        n = h.numel()
        if n % bs != 0 or n // bs < 2:
            raise ValueError("batch of %d triples does not match batch_size %d with negatives" % (n, bs))
        neg = n // bs - 1
        out = torch.zeros(1, dtype=torch.float32, device=dev)
        _native.check(_native.lib().pt_trainer_step(self._native, None, bs, neg, 0, 0, _native.ptr(h),
                                                    _native.ptr(t), _native.ptr(r), _native.ptr(out),
                                                    _native.stream()))
        return out.item()

    def _run_batches(self, L, sampler, bern, bs, nb, losses, buf):
        """One epoch of device-sampled batches outside the fused form - cross sampling (the loader's
        __iter__ alternates tail_batch / head_batch, TrainDataLoader.py:240-246, 320-324) or relation
        corruption (neg_rel > 0): every batch is drawn by the GPU sampler into device arrays (k_sample,
        bit-identical to the loader's sampling call) and trained by the external-batch step."""
        dl = self.data_loader
        neg, neg_rel = dl.negative_ent, dl.negative_rel
        h, t, r, y = buf
        st = _native.stream()
        for i in range(nb):
            if dl.sampling_mode == "normal":
                mode = 0
            else:
                dl.cross_sampling_flag = 1 - dl.cross_sampling_flag
                mode = -1 if dl.cross_sampling_flag == 0 else 1
            _native.check(L.pt_sampler_sample_ex(sampler, bs, neg, neg_rel, mode, bern, dl.filter, _native.ptr(h),
                                                 _native.ptr(t), _native.ptr(r), _native.ptr(y), st))
            if mode != 0:
                # sampling_head / sampling_tail hand the model only the first bs relations and fixed-side
                # entities (TrainDataLoader.py:212-217, :231-236) and TransE/TransH broadcast them over every
                # negative (TransE.py:51-58): a relation-corruption slot trains as a copy of its positive
                fixed = t if mode == -1 else h
                fixed.view(-1, bs)[1:] = fixed[:bs]
                r.view(-1, bs)[1:] = r[:bs]
            _native.check(L.pt_trainer_step(self._native, None, bs, neg + neg_rel, 0, 0, _native.ptr(h),
                                            _native.ptr(t), _native.ptr(r), _native.ptr(losses[i:i + 1]), st))

    def run(self):
        ns, kge, loss = self._setup()
        dl = self.data_loader
        bs, nb, neg = dl.batch_size, dl.nbatches, dl.negative_ent
        if ns.batch_size != bs:
            raise ValueError("NegativeSampling.batch_size (%d) differs from the loader's (%d)" % (ns.batch_size, bs))
        L = _native.lib()
        sampler = dl.device_sampler()
        bern = L.pt_legacy_bern()
        dev = kge.ent_embeddings.weight.device
        losses = torch.zeros(max(nb, 1), dtype=torch.float32, device=dev)
        fused = dl.sampling_mode == "normal" and dl.negative_rel == 0
        buf = None
        if not fused:
            seq = bs * (1 + neg + dl.negative_rel)
            buf = tuple(torch.zeros(seq, dtype=torch.int64, device=dev) for _ in range(3)) + \
                (torch.zeros(seq, dtype=torch.float32, device=dev),)
        print("Finish initializing...")
        training_range = tqdm(range(self.train_times))
        for epoch in training_range:
            if nb > 0 and fused:
                _native.check(L.pt_trainer_run(self._native, sampler, bs, neg, bern, dl.filter, nb,
                                               _native.ptr(losses), _native.stream()))
            elif nb > 0:
                losses.zero_()
                self._run_batches(L, sampler, bern, bs, nb, losses, buf)
            host = losses.cpu().numpy()
            self.last_step_losses = host[:nb].copy()
            res = float(host[:nb].sum())
            loss_v = float(host[nb - 1]) if nb > 0 else 0.0
            training_range.set_description("Epoch %d | loss: %f" % (epoch, loss_v))
            if self.save_steps and self.checkpoint_dir and (epoch + 1) % self.save_steps == 0:
                print("Epoch %d has finished, saving..." % (epoch))
                kge.save_checkpoint(os.path.join(self.checkpoint_dir + "-" + str(epoch) + ".ckpt"))
        self.last_epoch_loss = res if self.train_times > 0 else 0.0

    def set_model(self, model):
        self.model = model

    def to_var(self, x, use_gpu):
        return torch.from_numpy(x).cuda()

    def set_use_gpu(self, use_gpu):
        self.use_gpu = use_gpu

    def set_alpha(self, alpha):
        self.alpha = alpha
        if self.optimizer is not None:
            self.optimizer.lr = alpha

    def set_lr_decay(self, lr_decay):
        self.lr_decay = lr_decay

    def set_weight_decay(self, weight_decay):
        self.weight_decay = weight_decay

    def set_opt_method(self, opt_method):
        self.opt_method = opt_method

    def set_train_times(self, train_times):
        self.train_times = train_times

    def set_save_steps(self, save_steps, checkpoint_dir=None):
        self.save_steps = save_steps
        if not self.checkpoint_dir:
            self.set_checkpoint_dir(checkpoint_dir)

    def set_checkpoint_dir(self, checkpoint_dir):
        self.checkpoint_dir = checkpoint_dir

    def set_deterministic(self, deterministic):
        self.deterministic = bool(deterministic)
