import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import _native
from .Model import Model


class TransE(Model):
    """TransE (openke/module/model/TransE.py:8-93): same constructor, parameters and initialisation
    (nn.Embedding, then xavier_uniform_ from the torch generator, :17-36). Scores come from the HIP
    scoring kernel; training from the fused step kernels driven by openke.config.Trainer."""

    native_model = _native.PT_TRANSE

    def __init__(self, ent_tot, rel_tot, dim=100, p_norm=1, norm_flag=True, margin=None, epsilon=None):
        super(TransE, self).__init__(ent_tot, rel_tot)
        self.dim = dim
        self.margin = margin
        self.epsilon = epsilon
        self.norm_flag = norm_flag
        self.p_norm = p_norm
        self.ent_embeddings = self._embedding(self.ent_tot, self.dim)
        self.rel_embeddings = self._embedding(self.rel_tot, self.dim)
        if margin is None or epsilon is None:
            self._xavier_uniform_(self.ent_embeddings.weight.data)
            self._xavier_uniform_(self.rel_embeddings.weight.data)
        else:
            self.embedding_range = nn.Parameter(torch.Tensor([(self.margin + self.epsilon) / self.dim]),
                                                requires_grad=False)
            self._uniform_(self.ent_embeddings.weight.data, -self.embedding_range.item(), self.embedding_range.item())
            self._uniform_(self.rel_embeddings.weight.data, -self.embedding_range.item(), self.embedding_range.item())
        if margin is not None:
            self.margin = nn.Parameter(torch.Tensor([margin]))
            self.margin.requires_grad = False
            self.margin_flag = True
        else:
            self.margin_flag = False

    def _calc(self, h, t, r, mode):
        """Tensor-level score of given embedding rows (TransE.py:46-60); used by the null-vector tuple
        scores of Parallel_Universe_Config, not by the training or ranking hot path."""
        if self.norm_flag:
            h = F.normalize(h, 2, -1)
            r = F.normalize(r, 2, -1)
            t = F.normalize(t, 2, -1)
        if mode != 'normal':
            h = h.view(-1, r.shape[0], h.shape[-1])
            t = t.view(-1, r.shape[0], t.shape[-1])
            r = r.view(-1, r.shape[0], r.shape[-1])
        if mode == 'head_batch':
            score = h + (r - t)
        else:
            score = (h + r) - t
        return torch.norm(score, self.p_norm, -1).flatten()

    def forward(self, data):
        score = self.native_score(data)
        if self.margin_flag:
            return self.margin - score
        return score

    def regularization(self, data):
        raise NotImplementedError("regularisation is outside the accelerated path (regul_rate is 0 in every config)")

    def predict(self, data):
        score = self.forward(data)
        if self.margin_flag:
            score = self.margin - score
        return score.cpu().data.numpy()
