import torch
import torch.nn as nn
import torch.nn.functional as F

from .Loss import Loss


class MarginLoss(Loss):
    """mean(max(p - n, -margin)) + margin (openke/module/loss/MarginLoss.py:24-28). In training the
    value and its gradient are computed inside the fused HIP step; forward() here evaluates the same
    expression on given score tensors (value only)."""

    def __init__(self, adv_temperature=None, margin=6.0):
        super(MarginLoss, self).__init__()
        self.margin = nn.Parameter(torch.Tensor([margin]))
        self.margin.requires_grad = False
        if adv_temperature is not None:
            self.adv_temperature = nn.Parameter(torch.Tensor([adv_temperature]))
            self.adv_temperature.requires_grad = False
            self.adv_flag = True
        else:
            self.adv_flag = False

    def get_weights(self, n_score):
        return F.softmax(-n_score * self.adv_temperature, dim=-1).detach()

    def forward(self, p_score, n_score):
        if self.adv_flag:
            return (self.get_weights(n_score) * torch.max(p_score - n_score, -self.margin)).sum(dim=-1).mean() + \
                self.margin
        return (torch.max(p_score - n_score, -self.margin)).mean() + self.margin

    def predict(self, p_score, n_score):
        score = self.forward(p_score, n_score)
        return score.cpu().data.numpy()
