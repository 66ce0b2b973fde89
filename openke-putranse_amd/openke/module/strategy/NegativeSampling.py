from .Strategy import Strategy


class NegativeSampling(Strategy):
    """Positive/negative reshaping + loss (openke/module/strategy/NegativeSampling.py:5-31).
    Trainer.run never calls forward(): the fused HIP step computes this loss and its gradient in one
    pass. forward() remains for API use and returns the loss value (no autograd graph)."""

    def __init__(self, model=None, loss=None, batch_size=256, regul_rate=0.0, l3_regul_rate=0.0):
        super(NegativeSampling, self).__init__()
        self.model = model
        self.loss = loss
        self.batch_size = batch_size
        self.regul_rate = regul_rate
        self.l3_regul_rate = l3_regul_rate

    def _get_positive_score(self, score):
        positive_score = score[:self.batch_size]
        positive_score = positive_score.view(-1, self.batch_size).permute(1, 0)
        return positive_score

    def _get_negative_score(self, score):
        negative_score = score[self.batch_size:]
        negative_score = negative_score.view(-1, self.batch_size).permute(1, 0)
        return negative_score

    def forward(self, data):
        if self.regul_rate != 0 or self.l3_regul_rate != 0:
            raise NotImplementedError("regularisation is outside the accelerated path")
        score = self.model(data)
        p_score = self._get_positive_score(score)
        n_score = self._get_negative_score(score)
        return self.loss(p_score, n_score)
