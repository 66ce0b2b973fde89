# coding:utf-8
"""Validator (mirror of openke/config/Validator.py:18-56): filtered hit@10 of the validation split for
the early-stopping loops of the reference's static experiments (experiments/static_experiment_*.py).

valid() is validInit + validHead/validTail over every validation triple + getValidHit10 (Valid.h:38-44,
:117-256): the scores of all validation queries come from the GPU scoring kernel (pt_score_rows) and
their filtered ranks from pt_rank_rows - the same counts as validHead/validTail on the candidate-order
vectors - and hit@10 with the reference's float arithmetic: per side #{filtered rank < 10} / validTotal,
then their mean."""
import numpy as np

from .Tester import Tester


class Validator(Tester):
    def __init__(self, model=None, data_loader=None):
        super(Validator, self).__init__(data_loader=data_loader, use_gpu=True)
        self.model = model
        if self.model is not None:
            self.model.cuda()
        self.valid_dataloader = data_loader
        self.early_stopping_patience = 10
        self.bad_counts = 0
        self.best_hit10 = 0

    def valid(self):
        dl = self.valid_dataloader
        h, t, r = dl.eval_triples()
        n = np.float32(max(len(h), 1))
        ranks = self._rank_all(h, t, r, dl.get_ent_tot())
        self.last_ranks = tuple(ranks[:4])
        _, fh, _, ft = self.last_ranks
        l_tot = np.float32(np.count_nonzero(fh < 10)) / n
        r_tot = np.float32(np.count_nonzero(ft < 10)) / n
        return float((l_tot + r_tot) / np.float32(2))

    def valid_one_step(self, data):
        return self.model.predict(data)
