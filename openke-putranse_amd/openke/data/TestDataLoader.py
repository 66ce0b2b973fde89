# coding:utf-8
"""Evaluation data loader (mirror of openke/data/TestDataLoader.py of the reference): link-prediction
batches (sampling_lp) and triple-classification batches (sampling_tc: the test triples and one filtered
negative each from the library's getTestBatch, Test.h:576-599).

read() has the reference's side effects on the global context (re-seeding the sampler with its
random_seed, default 4, and re-importing the training set, TestDataLoader.py:276-290)."""
import ctypes

import numpy as np

from .. import _native


class TestDataSampler(object):

    def __init__(self, data_total, data_sampler):
        self.data_total = data_total
        self.data_sampler = data_sampler
        self.total = 0

    def __iter__(self):
        return self

    def __next__(self):
        self.total += 1
        if self.total > self.data_total:
            raise StopIteration()
        return self.data_sampler()

    def __len__(self):
        return self.data_total


class TestDataLoader(object):

    def __init__(self, in_path="./", sampling_mode='link', random_seed=4, mode='test', setting="static",
                 load_all_triples=False, count_header=None):
        self.lib = _native.lib()
        if setting != "static":
            raise NotImplementedError("only the static setting is part of the accelerated path")
        self.setting = setting
        self.mode = mode
        self.load_all_triples = load_all_triples
        self.in_path = in_path
        self.sampling_mode = sampling_mode
        self.random_seed = random_seed
        # see TrainDataLoader. None (default): the file format the process already reads with - the train
        # loader's choice - so a TrainDataLoader(count_header=True) followed by a default TestDataLoader does
        # not make importTrainFiles see a format change and re-read train2id.txt under the other format
        self.count_header = None if count_header is None else bool(count_header)
        self.read()

    def set_path(self, in_path):
        self.lib.setInPath(ctypes.create_string_buffer(in_path.encode(), len(in_path) * 2))

    def read(self):
        self.set_path(self.in_path)
        if self.count_header is None:
            self.count_header = bool(self.lib.pt_get_count_header())
        _native.check(self.lib.pt_set_count_header(1 if self.count_header else 0))
        self.lib.setRandomSeed(self.random_seed)
        self.lib.randReset()
        self.lib.importTrainFiles()
        _native.check(self.lib.pt_legacy_import_status())
        if self.load_all_triples:
            self.lib.activateLoadOfAllTriples(1)
        self.lib.importTestFiles()
        _native.check(self.lib.pt_legacy_import_status())
        self.relTotal = self.lib.getRelationTotal()
        self.entTotal = self.lib.getEntityTotal()
        E = self.entTotal
        if self.mode == 'test':
            self.testTotal = self.lib.getTestTotal()
            self.test_h = np.zeros(E, dtype=np.int64)
            self.test_t = np.zeros(E, dtype=np.int64)
            self.test_r = np.zeros(E, dtype=np.int64)
            n = self.testTotal
            self.test_pos_h, self.test_pos_t, self.test_pos_r = (np.zeros(n, dtype=np.int64) for _ in range(3))
            self.test_neg_h, self.test_neg_t, self.test_neg_r = (np.zeros(n, dtype=np.int64) for _ in range(3))
        elif self.mode == 'valid':
            self.validTotal = self.lib.getValidTotal()
            self.valid_h = np.zeros(E, dtype=np.int64)
            self.valid_t = np.zeros(E, dtype=np.int64)
            self.valid_r = np.zeros(E, dtype=np.int64)

    @staticmethod
    def _addr(a):
        return a.__array_interface__["data"][0]

    def sampling_lp(self):
        res = []
        if self.mode == 'test':
            h, t, r = self.test_h, self.test_t, self.test_r
            head_fn, tail_fn = self.lib.getHeadBatch, self.lib.getTailBatch
        else:
            h, t, r = self.valid_h, self.valid_t, self.valid_r
            head_fn, tail_fn = self.lib.getValidHeadBatch, self.lib.getValidTailBatch
        head_fn(self._addr(h), self._addr(t), self._addr(r))
        res.append({"batch_h": h.copy(), "batch_t": t[:1].copy(), "batch_r": r[:1].copy(), "mode": "head_batch"})
        tail_fn(self._addr(h), self._addr(t), self._addr(r))
        res.append({"batch_h": h[:1], "batch_t": t, "batch_r": r[:1], "mode": "tail_batch"})
        return res

    def sampling_tc(self):
        """TestDataLoader.py:186-205: every test triple and one negative (the same buffers each call)."""
        if self.mode != 'test':
            raise NotImplementedError("triple classification samples the test split (the reference's only mode)")
        self.lib.getTestBatch(self._addr(self.test_pos_h), self._addr(self.test_pos_t), self._addr(self.test_pos_r),
                              self._addr(self.test_neg_h), self._addr(self.test_neg_t), self._addr(self.test_neg_r))
        return [
            {"batch_h": self.test_pos_h, "batch_t": self.test_pos_t, "batch_r": self.test_pos_r, "mode": "normal"},
            {"batch_h": self.test_neg_h, "batch_t": self.test_neg_t, "batch_r": self.test_neg_r, "mode": "normal"},
        ]

    def eval_triples(self):
        """(h, t, r) int64 arrays of this loader's split in the reference's ranking order."""
        valid = 1 if self.mode == 'valid' else 0
        n = self.lib.pt_legacy_eval_triples(valid, None, None, None)
        h, t, r = (np.zeros(n, dtype=np.int64) for _ in range(3))
        self.lib.pt_legacy_eval_triples(valid, self._addr(h), self._addr(t), self._addr(r))
        return h, t, r

    """interfaces to get essential parameters"""

    def get_ent_tot(self):
        return self.entTotal

    def get_rel_tot(self):
        return self.relTotal

    def get_triple_tot(self):
        return self.testTotal

    def set_sampling_mode(self, sampling_mode):
        self.sampling_mode = sampling_mode

    def __len__(self):
        return self.testTotal if self.mode == 'test' else self.validTotal

    def __iter__(self):
        if self.sampling_mode == 'link':
            if self.mode == 'test':
                self.lib.initTest()
                eval_total = self.testTotal
            else:
                self.lib.validInit()
                eval_total = self.validTotal
            return TestDataSampler(eval_total, self.sampling_lp)
        self.lib.initTest()
        return TestDataSampler(1, self.sampling_tc)
