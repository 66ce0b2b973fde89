# coding:utf-8
"""PuTransE / PuTransH driver (mirror of openke/config/Parallel_Universe_Config.py).

Same constructor, attributes, per-universe protocol and outputs as the reference; the work is
re-organised for the GPU:

* Training. The reference builds and trains universes one at a time (train_parallel_universes,
  :316-367). Universe k is a pure function of seed0 + k (set_random_seed, :157-161), so here a WAVE of
  universes is prepared at once - the Python draws of every universe in the reference's order
  (randrange(tc), uniform(balance), randrange(margin), randrange(epochs), uniform(lr); :210-236), the
  universe construction on host threads (pt_universe_build_many; getParallelUniverse), the torch init
  of every universe's tables after torch.manual_seed(seed0 + k) (the model factory, :169-177) - and
  the whole wave trains in ONE persistent GPU launch (pt_universes_train: one workgroup per universe
  runs all of its epochs x nbatches Adagrad steps, :238-258). The universes are then committed one by
  one in id order with the reference's validation / early-stopping / checkpoint schedule; universes a
  wave trained beyond an early stop are discarded, so the committed result is the reference's.
* Multi-GPU. With torch.distributed initialised (one process per GPU), universe k trains on rank
  k % world_size (universes are independent: no data-path collective). Link-prediction score rows
  are MIN-combined across ranks with one all_reduce(MIN) over RCCL.
* Global energy estimation. The per-(entity, relation) score dictionaries (:446-465, :516-554) are
  device rows [n_keys][entTotal] filled by pt_lp_min_scores (score every entity of every universe
  holding the key, MIN into the key row); ranks come from pt_rank_rows on those rows (the same counts
  as testHead/testTail and validHead/validTail on the candidate-order vectors), metrics from
  pt_lp_metrics.
"""
import ctypes
import gc
import os
import pickle
import random
import sys
import threading
import time
from collections import defaultdict
from copy import copy, deepcopy
from random import randrange, uniform, seed

import numpy as np
import torch

from .. import _native
from . import _checkpoint, _map_pickle
from ..data import TestDataLoader
from ..module.loss import MarginLoss
from ..module.model.Model import Model
from ..module.strategy import NegativeSampling
from .Tester import Tester, device_type_lists, rank_types


def get_string_key(entity, relation):
    return '{},{}'.format(entity, relation)


def defaultdict_int(innerfactory=int):
    return defaultdict(innerfactory)


def float_default():
    return float("inf")


def to_tensor(x, use_gpu):
    if use_gpu:
        return torch.tensor([x]).cuda()
    return torch.tensor([x])


def _dist():
    """(world_size, rank) of an initialised torch.distributed group, else (1, 0)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def universe_owner(universe_id, world_size):
    """Round-robin rank of universe `universe_id`: the owner of a universe no placement map names
    (universes committed through add_universe / the one-universe protocol)."""
    return universe_id % world_size


def universe_cost(epochs, triples, dim):
    """Relative GPU time of training one universe: epochs x training triples (the slot count up to the
    constant nbatches / negative factors) times the per-slot row work, dim floats per embedding row plus
    ~32 floats' worth of fixed per-slot sampling / loss work (the universes kernel's step profile)."""
    return float(max(epochs, 0)) * float(max(triples, 0)) * (float(dim) + 32.0)


def place_universes(costs, world_size, loads=None):
    """LPT placement (longest processing time first) of independent universes over ranks: universes in
    decreasing cost (ties by id) each go to the rank with the least cost so far (ties to the lowest
    rank). `costs` maps universe id -> cost; returns {universe id: rank}. `loads` (optional, one float per
    rank) is the cost each rank already carries - earlier training waves - and is updated in place, so
    consecutive waves balance the whole run instead of each wave starting from zero (which would give
    rank 0 the heaviest universe of every wave, and every universe of one-universe waves). A pure function
    of its arguments, so every rank computes the same map from the same draws with no communication."""
    if loads is None:
        loads = [0.0] * max(int(world_size), 1)
    if len(loads) != max(int(world_size), 1):
        raise ValueError("place_universes: %d loads for %d ranks" % (len(loads), world_size))
    owners = {}
    for uid, c in sorted(costs.items(), key=lambda kv: (-kv[1], kv[0])):
        r = min(range(len(loads)), key=lambda i: (loads[i], i))
        owners[uid] = r
        loads[r] += c
    return owners


def min_combine(tensors):
    """Element-wise MIN of the same tensors across all ranks (RCCL all_reduce(MIN) on the GPU path,
    gloo on CPU); no-op on one process. The global energy of a key is the min over every universe,
    whichever rank trained it (Parallel_Universe_Config.py:516-543)."""
    world, _ = _dist()
    if world > 1:
        import torch.distributed as dist
        host = dist.get_backend() != "nccl"   # gloo reduces host tensors (RCCL reduces in HBM over xGMI)
        for t in tensors:
            if host and t.is_cuda:
                h = t.cpu()
                dist.all_reduce(h, op=dist.ReduceOp.MIN)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return tensors


def lookup_local(sorted_global, order, query):
    """Local ids of global ids `query` in a universe given its sorted global ids and their local ids
    (-1 where absent)."""
    query = np.asarray(query, dtype=np.int64)
    if len(sorted_global) == 0:
        return np.full(len(query), -1, dtype=np.int64)
    pos = np.searchsorted(sorted_global, query)
    pos = np.minimum(pos, len(sorted_global) - 1)
    hit = sorted_global[pos] == query
    return np.where(hit, order[pos], -1)


def lp_pairs(slot, ent_remap, rel_remap, key_anchor, key_rel, key_side):
    """(key, universe slot, local anchor, local relation, side) for every evaluation key whose anchor
    entity AND relation the universe holds - the universes eval_universes scores for that key
    (Parallel_Universe_Config.py:470-476)."""
    em = np.asarray(ent_remap, dtype=np.int64)
    rm = np.asarray(rel_remap, dtype=np.int64)
    eo = np.argsort(em, kind="stable")
    ro = np.argsort(rm, kind="stable")
    la = lookup_local(em[eo], eo, key_anchor)
    lr = lookup_local(rm[ro], ro, key_rel)
    sel = np.nonzero((la >= 0) & (lr >= 0))[0]
    # int32 [n][5] rows, the memory layout of pt_lp_pair (key, universe, anchor, rel, side)
    out = np.empty((len(sel), 5), dtype=np.int32)
    out[:, 0] = sel
    out[:, 1] = slot
    out[:, 2] = la[sel]
    out[:, 3] = lr[sel]
    out[:, 4] = np.asarray(key_side)[sel]
    return out


def lp_pairs_all(ent_remaps, rel_remaps, key_anchor, key_rel, key_side):
    """lp_pairs of every universe slot at once (pt_lp_pairs: an inverted index of the universes' entities by
    global id joined with the keys, the relation looked up in each universe's sorted relations). Returns int32
    [n][5] rows (key, slot, local anchor, local relation, side), ordered by key then slot."""
    key_anchor = np.ascontiguousarray(key_anchor, dtype=np.int64)
    key_rel = np.ascontiguousarray(key_rel, dtype=np.int64)
    key_side = np.ascontiguousarray(key_side, dtype=np.int64)
    if not ent_remaps or len(key_anchor) == 0:
        return np.zeros((0, 5), dtype=np.int32)
    L = _native.lib()
    n = len(ent_remaps)
    eoff, roff = np.zeros(n + 1, dtype=np.int64), np.zeros(n + 1, dtype=np.int64)
    np.cumsum([len(m) for m in ent_remaps], out=eoff[1:])
    np.cumsum([len(m) for m in rel_remaps], out=roff[1:])
    eids = np.ascontiguousarray(np.concatenate(ent_remaps), dtype=np.int64)
    rids = np.ascontiguousarray(np.concatenate(rel_remaps), dtype=np.int64)
    cnt = np.zeros(1, dtype=np.int64)
    args = (n, eoff.ctypes.data, eids.ctypes.data, roff.ctypes.data, rids.ctypes.data, len(key_anchor),
            key_anchor.ctypes.data, key_rel.ctypes.data, key_side.ctypes.data)
    _native.check(L.pt_lp_pairs(*args, None, 0, cnt.ctypes.data))
    out = np.empty((int(cnt[0]), 5), dtype=np.int32)
    _native.check(L.pt_lp_pairs(*args, out.ctypes.data, len(out), cnt.ctypes.data))
    return out[:int(cnt[0])]


def lp_pair_array(parts):
    """Concatenated lp_pairs blocks as one C-contiguous int32 [n][5] array (pt_lp_pair layout) and the
    pointer pt_lp_min_scores takes."""
    if not parts:
        arr = np.zeros((0, 5), np.int32)
    else:   # (one block: no copy - C4's 2 M rows are 41 MB)
        arr = np.ascontiguousarray(parts[0] if len(parts) == 1 else np.concatenate(parts), dtype=np.int32)
    return arr, arr.ctypes.data_as(ctypes.POINTER(_native.LpPair))


class _KeyStore(object):
    """Device score rows of one evaluation split: one row per (side, anchor, relation) key.

    side 0 = head prediction, anchor = tail (evaluation_tail2head_triple_score_dict, key 't,r');
    side 1 = tail prediction, anchor = head (evaluation_head2tail_triple_score_dict, key 'h,r') - the
    side convention of every native entry point (pt_lp_min_scores, pt_rank_rows, pt_known_partners)."""

    def __init__(self, h, t, r, ent_tot, device):
        self.h, self.t, self.r = h, t, r
        self.E = ent_tot
        keys = {}
        self.q_row = [np.zeros(len(h), dtype=np.int64), np.zeros(len(h), dtype=np.int64)]
        for q in range(len(h)):
            for side, anchor in ((0, int(t[q])), (1, int(h[q]))):
                k = (side, anchor, int(r[q]))
                idx = keys.get(k)
                if idx is None:
                    idx = keys[k] = len(keys)
                self.q_row[side][q] = idx
        self.keys = keys
        n = len(keys)
        self.key_side = np.array([k[0] for k in keys], dtype=np.int64)
        self.key_anchor = np.array([k[1] for k in keys], dtype=np.int64)
        self.key_rel = np.array([k[2] for k in keys], dtype=np.int64)
        self.rows = torch.full((max(n, 1), max(ent_tot, 1)), float("inf"), dtype=torch.float32, device=device)
        self.tuple = torch.full((max(n, 1),), float("inf"), dtype=torch.float32, device=device)
        self.folded = 0   # universes [0, folded) are MIN-ed into the rows
        self.rank_inputs = {}   # (known-set handle, side) -> the split's device ranking inputs (_ranks)

    def row(self, side, anchor, rel):
        idx = self.keys.get((side, int(anchor), int(rel)))
        return None if idx is None else idx


class _ArrayOf(object):
    """Pickles as numpy.asarray(t): the ndarray over a CPU tensor's memory."""
    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t

    def __reduce__(self):
        return (np.asarray, (self.t,))


class _BytesOf(object):
    """Pickles as bytes(numpy.asarray(t)): the bytes of a uint8 tensor."""
    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t

    def __reduce__(self):
        return (bytes, (_ArrayOf(self.t),))


class _Pickled(object):
    """A checkpoint container serialized with the plain C pickler when wrapped (a snapshot: later changes
    to the container are not in it), or given as a ready pickle stream (_map_pickle), and restored as the
    container itself on load: pickle.loads(bytes(numpy.asarray(<uint8 tensor>))). torch.save's pickler calls its
    persistent-id hook once per object, ~1 s for C3's id maps alone (768k entries), and writes a bytes object
    through protocol 2's latin-1 text form (~14 ms per MB, 1.5x the size); the stream travels as a tensor storage
    instead (one raw record of the archive), rebuilt with torch's own tensor reconstruction and numpy / builtin
    callables only. The file's layout is unchanged: torch.load returns the plain dicts."""
    __slots__ = ("data",)

    def __init__(self, obj=None, stream=None):
        if stream is None:
            stream = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        self.data = torch.frombuffer(bytearray(stream), dtype=torch.uint8) if len(stream) else \
            torch.zeros(0, dtype=torch.uint8)

    def __reduce__(self):
        return (pickle.loads, (_BytesOf(self.data),))


def universe_dim(dim_param, uid):
    """Embedding dim of universe `uid`: `dim_param` as given (the reference's fixed dim), or - a build
    extension for BASELINE config C3 (dim ~ U{lo..hi} per universe) - a (lo, hi) pair, drawn from numpy's
    default_rng(1000 + uid) (a stream of its own: the reference's Python / torch / glibc draws are untouched)."""
    if isinstance(dim_param, (tuple, list)):
        lo, hi = int(dim_param[0]), int(dim_param[1])
        return int(np.random.default_rng(1000 + int(uid)).integers(lo, hi + 1))
    return int(dim_param)


def _id_map_property(name):
    """A reference attribute holding per-universe id maps (entity_id_mappings, ...): universes committed since
    the last read are registered first (_materialize_maps), in one batch."""
    def get(self):
        # the caller may change the dictionaries: from now on checkpoints pickle them as they are
        self.__dict__["_maps_exposed"] = True
        self._materialize_maps()
        return self.__dict__[name]

    def put(self, value):
        if name == "_entity_id_mappings":
            self.__dict__["_pending_maps"] = []   # a replaced state (load / best state) drops pending ones
        self.__dict__["_map_log"] = None   # dictionaries not built from registered universes alone
        self.__dict__[name] = value
    return property(get, put)


_MAP_KEYS = ('entity_id_mappings', 'relation_id_mappings', 'entity_universes', 'relation_universes')


class Parallel_Universe_Config(Tester):
    # the reference's dictionaries (universe -> global id -> local id, global id -> universes); filled lazily
    entity_id_mappings = _id_map_property("_entity_id_mappings")
    relation_id_mappings = _id_map_property("_relation_id_mappings")
    entity_universes = _id_map_property("_entity_universes")
    relation_universes = _id_map_property("_relation_universes")

    def __init__(self,
                 train_dataloader=None, training_identifier='', valid_dataloader=None, test_dataloader=None,
                 initial_num_universes=5000,
                 min_margin=1, max_margin=4, min_lr=0.01, max_lr=0.1, min_num_epochs=50, max_num_epochs=200,
                 const_num_epochs=None, min_triple_constraint=500, max_triple_constraint=2000, min_balance=0.25,
                 max_balance=0.5, embedding_model=None, embedding_model_param=None,
                 missing_embedding_handling='last_rank',
                 save_steps=5, checkpoint_dir='./checkpoint/', valid_steps=5, early_stopping_patience=5,
                 training_setting="static",
                 incremental_strategy="normal",
                 universe_wave_size=None, deterministic=False):
        super(Parallel_Universe_Config, self).__init__(data_loader=test_dataloader, use_gpu=torch.cuda.is_available())
        self._pending_maps = []           # (uid, ent_remap, rel_remap) committed, not yet in the dictionaries
        if training_setting != "static":
            raise NotImplementedError("the incremental setting is outside the accelerated path")

        """ Train data + variables"""
        self.train_dataloader = train_dataloader
        self.ent_tot = train_dataloader.entTotal
        self.rel_tot = train_dataloader.relTotal
        self.training_identifier = training_identifier

        """ "-constant traininghyper parameters" """
        self.embedding_model = embedding_model
        self.embedding_model_param = embedding_model_param

        """ Parallel Universe data structures """
        self.initial_num_universes = initial_num_universes
        self.next_universe_id = 0

        self.trained_embedding_spaces = defaultdict(Model)  # universe_id -> embedding_space
        self.entity_id_mappings = defaultdict(defaultdict_int)  # universe_id -> global entity_id -> local id
        self.relation_id_mappings = defaultdict(defaultdict_int)  # universe_id -> global relation_id -> local id

        self.entity_universes = defaultdict(set)  # entity_id -> universe_id
        self.relation_universes = defaultdict(set)  # relation_id -> universe_id
        # (uid, ent_remap, rel_remap) of every universe registered since the dictionaries were created: while
        # nothing else wrote them (no load / best state) and no caller read them, the checkpoint pickles them from
        # these arrays (_map_pickle) instead of materialising and pickling the dictionaries
        self._map_log = []
        self._maps_exposed = False

        self.initial_random_seed = self.train_dataloader.lib.getRandomSeed()

        """Parallel Universe spans for randomizing embedding space hyper parameters"""
        self.min_margin = min_margin
        self.max_margin = max_margin
        self.min_lr = min_lr
        self.max_lr = max_lr
        self.min_num_epochs = min_num_epochs
        self.max_num_epochs = max_num_epochs
        self.const_num_epochs = const_num_epochs
        self.min_triple_constraint = min_triple_constraint
        self.max_triple_constraint = max_triple_constraint
        self.min_balance = min_balance
        self.max_balance = max_balance

        """ saving """
        self.save_steps = save_steps
        self.checkpoint_dir = checkpoint_dir

        """ Eval """
        self.missing_embedding_handling = missing_embedding_handling  # "last_rank" | "null_vector"

        """ ""Valid"" """
        self.valid_dataloader = valid_dataloader if valid_dataloader is not None else TestDataLoader(
            train_dataloader.in_path,
            sampling_mode="link",
            mode='valid')

        self.valid_steps = valid_steps
        self.early_stopping_patience = early_stopping_patience
        self.early_stopping_patience_const = early_stopping_patience
        self.bad_counts = 0
        self.best_hit10 = 0
        self.best_state = None

        """Global Energy Estimation data structures"""
        self.current_tested_universes = 0
        self.current_validated_universes = 0
        # the reference's score dictionaries are device rows here (see _KeyStore); these stay empty
        self.evaluation_head2tail_triple_score_dict = {}
        self.evaluation_tail2head_triple_score_dict = {}
        self.evaluation_head2rel_tuple_score_dict = {}
        self.evaluation_tail2rel_tuple_score_dict = {}
        self.default_scores = None   # the reference's [inf] * entTotal template, not needed with device rows

        self.training_setting = training_setting
        self.incremental_strategy = incremental_strategy

        """ MI355X build """
        self.universe_wave_size = universe_wave_size
        # reference-order mode (ordered.hip): every universe's per-row gradient sums in slot order,
        # bit-identical run to run; the default fast kernel sums them in arrival order
        self.deterministic = bool(deterministic)
        self.last_universe_losses = {}    # universe_id -> per-epoch loss sums of Trainer.run
        self.universe_hparams = {}        # universe_id -> tc, balance, margin, epochs, lr, batch_size
        self._stores = {}                 # 'test' / 'valid' -> _KeyStore
        self._remap_cache = {}            # universe_id -> (ent_remap, rel_remap, sorted helpers)
        self._dev_remaps = {}             # universe_id -> device int64 local -> global entity map
        # multi-GPU: universe_id -> rank that trains / holds it (place_universes per training wave, re-made
        # by load_parameters for the loading job's world size); ids absent here are round-robin
        self.universe_owners = {}
        self._rank_loads = []             # per rank: cost of the universes placed on it so far (all waves)

    # ------------------------------------------------------------------ reference API -----------
    def get_default_value_list(self):
        return [float("inf") for i in range(self.ent_tot)]

    def set_min_max_triple_constraint(self, min, max):
        self.min_triple_constraint = min
        self.max_triple_constraint = max

    def set_random_seed(self, rand_seed):
        self.train_dataloader.lib.setRandomSeed(rand_seed)
        self.train_dataloader.lib.randReset()
        seed(rand_seed)
        torch.manual_seed(rand_seed)

    def set_valid_dataloader(self, valid_dataloader):
        self.valid_dataloader = valid_dataloader
        self._stores.pop('valid', None)

    def set_test_dataloader(self, test_dataloader):
        self.data_loader = test_dataloader
        self._stores.pop('test', None)

    def embedding_model_factory(self, ent_tot, rel_tot, margin):
        embedding_method = self.embedding_model(ent_tot, rel_tot, **self._model_param(self.next_universe_id))
        return NegativeSampling(
            model=embedding_method,
            loss=MarginLoss(margin=margin),
            batch_size=self.train_dataloader.batch_size
        )

    def reset_valid_variables(self):
        self.early_stopping_patience = self.early_stopping_patience_const
        self.best_state = {}
        self.best_hit10 = 0
        self.bad_counts = 0

    def add_embedding_space(self, embedding_space):
        for param in embedding_space.parameters():
            param.requires_grad = False
        self.trained_embedding_spaces[self.next_universe_id] = embedding_space

    def owner(self, uid):
        """Rank holding universe `uid` in this job."""
        world, _ = _dist()
        return self.universe_owners.get(uid, universe_owner(uid, world))

    # ------------------------------------------------------------------ training ----------------
    def _batched(self):
        """The multi-universe kernel draws normal-mode entity corruptions; cross sampling or relation
        corruption train universe by universe (the reference's protocol on the fused trainer)."""
        dl = self.train_dataloader
        return dl.sampling_mode == "normal" and dl.negative_rel == 0

    def _check_setup(self):
        if self.embedding_model is None or getattr(self.embedding_model, "native_model", None) is None:
            raise NotImplementedError("embedding_model must be openke.module.model.TransE or TransH")
        _native.require_gpu()

    def _universe_draws(self, uid):
        """Python-RNG draws of universe uid in the reference's order (:210-236): set_random_seed(seed0 + uid)
        seeds Python's generator, then randrange(tc), uniform(balance), randrange(margin), randrange(epochs),
        uniform(lr). Drawn from a private random.Random(seed0 + uid) - the same numbers - so a wave's draws need
        no global reseeding per universe (_train_wave reseeds the globals once, after the wave)."""
        rs = random.Random(self.initial_random_seed + uid)
        tc = rs.randrange(self.min_triple_constraint, self.max_triple_constraint)
        balance = round(rs.uniform(self.min_balance, self.max_balance), 2)
        margin = rs.randrange(self.min_margin, self.max_margin)
        epochs = self.const_num_epochs if self.const_num_epochs is not None \
            else rs.randrange(self.min_num_epochs, self.max_num_epochs)
        lr = round(rs.uniform(self.min_lr, self.max_lr), len(str(self.min_lr).split('.')[1]))
        return tc, balance, margin, epochs, lr

    def _model_param(self, uid):
        """embedding_model_param of universe uid (a (lo, hi) dim resolved per universe: universe_dim)."""
        param = dict(self.embedding_model_param)
        if "dim" in param:
            param["dim"] = universe_dim(param["dim"], uid)
        return param

    def _train_wave(self, ids):
        """Build and train universes `ids` (this rank's share on the GPU); returns records in id order.
        self.last_wave_timing: seconds spent in the Python draws, the native universe construction, the torch
        modules (factory init, owned universes only), their H2D copy, the GPU training launch (job setup,
        kernel, loss readback), per wave."""
        L = _native.lib()
        dl = self.train_dataloader
        world, rank = _dist()
        n = len(ids)
        tm = {"wave_universes": n}
        t0 = time.perf_counter()
        draws = [self._universe_draws(uid) for uid in ids]
        seeds = np.array([self.initial_random_seed + uid for uid in ids], dtype=np.int64)
        tcs = np.array([d[0] for d in draws], dtype=np.int64)
        bals = np.array([d[1] for d in draws], dtype=np.float32)
        handles = (ctypes.c_void_p * max(n, 1))()
        graph = L.pt_legacy_graph()
        if not graph:
            raise RuntimeError("no training graph imported (TrainDataLoader.read() imports it)")
        t1 = time.perf_counter()
        tm["draws_s"] = t1 - t0
        _native.check(L.pt_universe_build_many(graph, n, seeds.ctypes.data, dl.work_threads, tcs.ctypes.data,
                                               bals.ctypes.data, 0, handles))
        t0 = time.perf_counter()
        tm["native_build_s"] = t0 - t1
        recs, jobs, keep = [], [], []
        dev = torch.device("cuda", torch.cuda.current_device())
        tm["modules_s"] = tm["h2d_s"] = 0.0
        try:
            dims = [universe_dim(self.embedding_model_param.get("dim", 100), uid) for uid in ids]
            if world > 1:   # LPT over the wave from the draws and the built universes' sizes (same on every rank)
                if len(self._rank_loads) != world:
                    self._rank_loads = [0.0] * world
                self.universe_owners.update(place_universes(
                    {uid: universe_cost(draws[i][3], L.pt_universe_train_total(handles[i]), dims[i])
                     for i, uid in enumerate(ids)}, world, self._rank_loads))
            sizes = []
            for i, uid in enumerate(ids):
                tc, balance, margin, epochs, lr = draws[i]
                h = handles[i]
                E_u, R_u = L.pt_universe_ent_total(h), L.pt_universe_rel_total(h)
                N_u = L.pt_universe_train_total(h)
                em = np.zeros(max(E_u, 1), dtype=np.int64)
                rm = np.zeros(max(R_u, 1), dtype=np.int64)
                _native.check(L.pt_universe_remaps(h, em.ctypes.data, rm.ctypes.data))
                bs = N_u // dl.nbatches
                recs.append({"id": uid, "kge": None, "ent_remap": em[:E_u], "rel_remap": rm[:R_u], "tc": tc,
                             "balance": balance, "margin": margin, "epochs": epochs, "lr": lr, "batch_size": bs,
                             "train_total": N_u, "losses": None})
                sizes.append((E_u, R_u))
            # the model factory after torch.manual_seed(seed0 + uid) (set_random_seed, :157-161) for the universes
            # this rank trains (placement never changes a universe's init): Model.seeded draws the same tables from
            # a private generator, so the wave's modules are built on a thread pool
            mine = [i for i, uid in enumerate(ids) if self.owner(uid) == rank]
            ta = time.perf_counter()
            if mine and self.embedding_model.device_init_ok(dev):
                # the same tables drawn on the GPU straight into device tensors (Model.device_seeded: torch's CPU
                # generator restated, one launch for the wave; checked bit-identical to seeded() once per process)
                built = self.embedding_model.device_seeded(
                    [(self.initial_random_seed + ids[i], sizes[i][0], sizes[i][1], self._model_param(ids[i]))
                     for i in mine], dev)
                tm["modules_s"] = time.perf_counter() - ta
                for i, kge in zip(mine, built):
                    recs[i]["kge"] = kge
                tm["h2d_s"] = 0.0
            else:
                def build(i):
                    return self.embedding_model.seeded(self.initial_random_seed + ids[i], sizes[i][0], sizes[i][1],
                                                       **self._model_param(ids[i]))
                if len(mine) > 1:
                    from concurrent.futures import ThreadPoolExecutor
                    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1, len(mine))) as ex:
                        built = list(ex.map(build, mine))
                else:
                    built = [build(i) for i in mine]
                tb = time.perf_counter()
                tm["modules_s"] = tb - ta
                for i, kge in zip(mine, built):
                    recs[i]["kge"] = kge.to(dev)
                tm["h2d_s"] = time.perf_counter() - tb
            # every owned universe's Adagrad state (zero-init, the tables' shapes) carved from one zeroed buffer:
            # one allocation and one fill for the wave instead of one per table
            acc_elems = sum(sum(x.numel() for x in recs[i]["kge"].tables() if x is not None) for i in mine)
            acc_buf = torch.zeros(max(acc_elems, 1), dtype=torch.float32, device=dev)
            acc_off = 0
            for i in mine:
                uid, rec, h = ids[i], recs[i], handles[i]
                tc, balance, margin, epochs, lr = draws[i]
                bs = rec["batch_size"]
                kge = rec["kge"]
                ent, rel, nv = kge.tables()
                accs = []
                for x in (ent, rel, nv):
                    if x is None:
                        accs.append(None)
                        continue
                    accs.append(acc_buf[acc_off:acc_off + x.numel()].view(x.shape))
                    acc_off += x.numel()
                accs = tuple(accs)
                st = np.zeros(dl.work_threads, dtype=np.uint64)
                _native.check(L.pt_universe_seeds(h, st.ctypes.data))
                j = _native.UniverseJob()
                j.graph = L.pt_universe_graph(h)
                j.seeds = st.ctypes.data
                j.threads = dl.work_threads
                j.batch_size = bs
                j.epochs = epochs if bs > 0 else 0
                j.nbatches = dl.nbatches
                j.neg = dl.negative_ent
                j.lr = lr
                j.margin = margin
                j.ent, j.rel, j.normv = (x.data_ptr() if x is not None else None for x in (ent, rel, nv))
                j.ent_acc, j.rel_acc, j.norm_acc = (x.data_ptr() if x is not None else None for x in accs)
                j.dim = ent.shape[1]
                jobs.append(j)
                keep.append((st, accs, rec))
            # the process-global generators as the last set_random_seed of the wave leaves them (:157-161)
            self.set_random_seed(self.initial_random_seed + ids[-1])
            t1 = time.perf_counter()
            tm["jobs_s"] = t1 - t0 - tm["modules_s"] - tm["h2d_s"]
            tm["trained_here"] = len(jobs)
            if jobs:
                kge0 = keep[0][2]["kge"]
                total_epochs = sum(int(j.epochs) for j in jobs)
                losses = torch.zeros(max(total_epochs, 1), dtype=torch.float32, device=dev)
                arr = (_native.UniverseJob * len(jobs))(*jobs)
                _native.check(L.pt_universes_train_ex(arr, len(jobs), kge0.native_model, int(kge0.p_norm),
                                                      1 if kge0.norm_flag else 0, _native.PT_ADAGRAD,
                                                      int(dl.bern), int(dl.filter),
                                                      _native.PT_DETERMINISTIC if self.deterministic else 0,
                                                      _native.ptr(losses), _native.stream()))
                lh = losses.cpu().numpy()
                off = 0
                for j, (_, _, rec) in zip(jobs, keep):
                    rec["losses"] = lh[off:off + int(j.epochs)].copy()
                    off += int(j.epochs)
            tm["train_launch_s"] = time.perf_counter() - t1
        finally:
            for i in range(n):
                if handles[i]:
                    L.pt_universe_free(handles[i])
        self.last_wave_timing = tm
        return recs

    def _register_maps(self, uid, ent_remap, rel_remap):
        """process_universe_mappings (:179-207) for universe uid: the GPU paths read the arrays (_remap_cache)
        at once; the reference's dictionaries get the universe at their next read (_materialize_maps)."""
        em = np.ascontiguousarray(ent_remap, dtype=np.int64)
        rm = np.ascontiguousarray(rel_remap, dtype=np.int64)
        self._pending_maps.append((uid, em, rm))
        if self.__dict__.get("_map_log") is not None:
            self._map_log.append((uid, em, rm))
        self._remap_cache[uid] = (em, rm)   # the sorted lookup helpers on first use (_remaps)

    def _materialize_maps(self):
        """Register the pending universes' maps in the reference's dictionaries, all at once: the per-universe
        maps built by dict.update (C loops), the id -> universes sets grouped by id over every pending universe
        (one set update per id instead of one add per (id, universe)); new ids enter in order of first
        appearance, as process_universe_mappings (:179-207) adds them one universe after another."""
        pend = self.__dict__.get("_pending_maps")
        if not pend:
            return
        self.__dict__["_pending_maps"] = []
        d = self.__dict__
        emaps, rmaps = d["_entity_id_mappings"], d["_relation_id_mappings"]
        for uid, em, rm in pend:
            el, rl = em.tolist(), rm.tolist()
            emaps[uid].update(zip(el, range(len(el))))
            rmaps[uid].update(zip(rl, range(len(rl))))
        for key, col in (("_entity_universes", 1), ("_relation_universes", 2)):
            target = d[key]
            ids = np.concatenate([p[col] for p in pend])
            us = np.repeat(np.array([p[0] for p in pend], dtype=np.int64), [len(p[col]) for p in pend])
            o = np.argsort(ids, kind="stable")
            ids, us = ids[o], us[o]
            keys, starts, counts = np.unique(ids, return_index=True, return_counts=True)
            first = np.argsort(o[starts], kind="stable")
            ul = us.tolist()
            for k, lo, c in zip(keys[first].tolist(), starts[first].tolist(), counts[first].tolist()):
                target[k].update(ul[lo:lo + c])

    def add_universe(self, embedding_space, ent_remap, rel_remap):
        """Register a trained universe as id next_universe_id: add_embedding_space +
        process_universe_mappings (:179-207) from its local -> global entity / relation maps.
        embedding_space is None for a universe trained on another rank."""
        uid = self.next_universe_id
        self._register_maps(uid, ent_remap, rel_remap)
        if embedding_space is not None:
            self.add_embedding_space(embedding_space)
        self.next_universe_id += 1
        return uid

    # ---------------------------------------------------- the reference's one-universe protocol --
    # train_parallel_universes builds and trains whole waves of universes in one GPU launch; these are
    # the reference's per-universe steps (:195-258) for callers that drive one universe at a time:
    #     set_random_seed(seed0 + k); compile_train_datset(); sp = train_embedding_space();
    #     add_embedding_space(sp); next_universe_id += 1
    # They use the Base.so-compatible global context (getParallelUniverse / swapHelpers / resetUniverse
    # in the library) and the fused single-model trainer on the swapped-in universe graph.
    def process_universe_mappings(self):
        """:195-207: the compiled universe's local -> global maps under next_universe_id."""
        em, rm = self.train_dataloader.get_universe_mappings()
        print('Entities are %d' % len(em))
        self._register_maps(self.next_universe_id, em, rm)

    def compile_train_datset(self):
        """:209-226: draw the triple constraint and balance, build the universe (getParallelUniverse)."""
        triple_constraint = randrange(self.min_triple_constraint, self.max_triple_constraint)
        balance_param = round(uniform(self.min_balance, self.max_balance), 2)
        print('universe information-------------------')
        print('--- num of training triples: %d' % triple_constraint)
        self.train_dataloader.compile_universe_dataset(triple_constraint, balance_param)
        self._compiled_draws = (triple_constraint, balance_param)
        self.process_universe_mappings()
        lib = self.train_dataloader.lib
        print('--- num of universe entities: %d' % lib.getEntityTotalUniverse())
        print('--- num of universe relations: %d' % lib.getRelationTotalUniverse())
        print('---------------------------------------')
        print('Train dataset for embedding space compiled.')

    def train_embedding_space(self):
        """:228-258: margin / epochs / lr draws, the model factory and an Adagrad Trainer run over the
        swapped-in universe (the fused GPU epoch on the library's sampler, whose graph follows swapHelpers)."""
        from .Trainer import Trainer
        self._check_setup()
        lib = self.train_dataloader.lib
        entity_total_universe = lib.getEntityTotalUniverse()
        relation_total_universe = lib.getRelationTotalUniverse()
        train_total_universe = lib.getTrainTotalUniverse()
        margin = randrange(self.min_margin, self.max_margin)
        model = self.embedding_model_factory(ent_tot=entity_total_universe, rel_tot=relation_total_universe,
                                             margin=margin)
        train_times = self.const_num_epochs if self.const_num_epochs is not None \
            else randrange(self.min_num_epochs, self.max_num_epochs)
        lr = round(uniform(self.min_lr, self.max_lr), len(str(self.min_lr).split('.')[1]))
        trainer = Trainer(model=model, data_loader=self.train_dataloader, train_times=train_times, alpha=lr,
                          use_gpu=True, opt_method='Adagrad', deterministic=self.deterministic)
        print('hyperparams for universe %d------------' % self.next_universe_id)
        print('--- epochs: %d' % train_times)
        print('--- learning rate:', lr)
        print('--- margin: %d' % margin)
        self.train_dataloader.swap_helpers()
        trainer.run()
        self.train_dataloader.reset_universe()
        self.universe_hparams[self.next_universe_id] = {
            "tc": getattr(self, "_compiled_draws", (None, None))[0],
            "balance": getattr(self, "_compiled_draws", (None, None))[1], "margin": margin, "epochs": train_times, "lr": lr,
            "batch_size": model.batch_size, "train_total": train_total_universe}
        return model.model

    def _commit(self, rec):
        assert rec["id"] == self.next_universe_id
        _, rank = _dist()
        uid = self.add_universe(rec["kge"] if self.owner(rec["id"]) == rank else None, rec["ent_remap"],
                                rec["rel_remap"])
        if rec["losses"] is not None:
            self.last_universe_losses[uid] = rec["losses"]
        self.universe_hparams[uid] = {k: rec[k] for k in ("tc", "balance", "margin", "epochs", "lr", "batch_size",
                                                         "train_total")}

    def _after_universe(self, universe_id):
        """Validation / early stopping / checkpoint schedule after universe `universe_id` of this call
        (Parallel_Universe_Config.py:329-365); True when training stops early."""
        tm = getattr(self, "last_train_timing", None)
        if (universe_id + 1) % self.valid_steps == 0:
            print("Universe %d has finished, validating..." % (self.next_universe_id - 1))
            t0 = time.perf_counter()
            self.eval_universes(eval_mode='valid')
            hit10 = self.valid()
            if tm is not None:
                tm["validations"] = tm.get("validations", 0) + 1
                tm["validate_s"] = tm.get("validate_s", 0.0) + time.perf_counter() - t0
            print("Current hit@10: {}".format(hit10))
            if hit10 > self.best_hit10:
                self.best_hit10 = hit10
                print("Best model | hit@10 of valid set is %f" % self.best_hit10)
                print('Save model at universe %d.' % self.next_universe_id)
                t0 = time.perf_counter()
                self.save_model("Best_model_Pu{}_{}.ckpt".format(self.embedding_model.__name__,
                                                                 self.training_identifier), background=True)
                if tm is not None:
                    tm["checkpoints"] = tm.get("checkpoints", 0) + 1
                    tm["checkpoint_s"] = tm.get("checkpoint_s", 0.0) + time.perf_counter() - t0
                self.bad_counts = 0
            else:
                print("Hit@10 of valid set is %f | bad count is %d" % (hit10, self.bad_counts))
                self.bad_counts += 1
            if self.bad_counts == self.early_stopping_patience:
                print("Early stopping at universe {}".format(self.next_universe_id - 1))
                self.get_best_state()
                return True
        if self.save_steps and self.checkpoint_dir and (universe_id + 1) % self.save_steps == 0:
            print('Save model at universe %d.' % self.next_universe_id)
            self.save_model()
        return False

    def train_parallel_universes(self, num_of_embedding_spaces):
        gc_was = gc.isenabled()
        ok = False
        try:
            self._train_parallel_universes(num_of_embedding_spaces, gc_was)
            ok = True
        finally:
            if gc_was:
                gc.enable()
            if not ok:   # a background checkpoint write still running: join it (and restore the switch interval)
                try:
                    self.flush_checkpoint()
                except Exception:
                    pass   # the training error is the one that propagates

    def _train_parallel_universes(self, num_of_embedding_spaces, gc_was=True):
        self._check_setup()
        training_duration = 0.0
        if not self._batched():
            # cross sampling / relation corruption: the reference's loop (:320-327), one universe at a time
            for universe_id in range(num_of_embedding_spaces):
                t0 = time.time()
                self.set_random_seed(self.initial_random_seed + self.next_universe_id)
                self.compile_train_datset()
                embedding_space = self.train_embedding_space()
                self.add_embedding_space(embedding_space)
                self.next_universe_id += 1
                training_duration += time.time() - t0
                if self._after_universe(universe_id):
                    break
            self.flush_checkpoint()
            print('Time took for creation of embedding spaces: {:5.3f}s'.format(training_duration), end='\n')
            return
        done = 0
        stop = False
        wave_size = self.wave_size()
        self.last_train_timing = timing = {"waves": 0, "universes": 0, "wave_s": 0.0, "commit_s": 0.0,
                                           "validate_save_s": 0.0}
        while done < num_of_embedding_spaces and not stop:
            # the cyclic collector paused for the wave: it creates tens of thousands of objects (modules, id maps),
            # enough to trigger full collections over everything the process holds in the middle of the loop;
            # collection runs again between waves
            gc.disable()
            wave = min(num_of_embedding_spaces - done, wave_size)
            ids = list(range(self.next_universe_id, self.next_universe_id + wave))
            t0 = time.time()
            recs = self._train_wave(ids)
            wave_s = time.time() - t0
            per_universe = wave_s / max(len(recs), 1)
            timing["waves"] += 1
            timing["wave_s"] += wave_s
            for k, v in self.last_wave_timing.items():
                timing[k] = timing.get(k, 0) + v
            print("trained universes %d..%d on the GPU (%.3f s)" % (ids[0], ids[-1], wave_s))
            for rec in recs:
                universe_id = done
                ta = time.time()
                self._commit(rec)
                tb = time.time()
                timing["commit_s"] += tb - ta
                training_duration += per_universe
                stop = self._after_universe(universe_id)
                timing["validate_save_s"] += time.time() - tb
                if stop:
                    break
                done += 1
                timing["universes"] += 1
            if gc_was:
                gc.enable()
        t0 = time.time()
        self.flush_checkpoint()
        timing["checkpoint_flush_s"] = time.time() - t0
        w = self.__dict__.pop("_ckpt_write_s", [])
        timing["checkpoint_writes"], timing["checkpoint_write_s"] = len(w), sum(w)
        print('Time took for creation of embedding spaces: {:5.3f}s'.format(training_duration), end='\n')

    def wave_size(self):
        """Universes per training launch: universe_wave_size if set, else a multiple of valid_steps of about
        512 per rank (two per CU of an MI355X: enough to fill the GPU), so an early stop - decided at a
        validation point - discards at most the rest of one wave."""
        if self.universe_wave_size:
            return max(int(self.universe_wave_size), 1)
        world, _ = _dist()
        vs = max(int(self.valid_steps or 1), 1)
        target = 512 * world
        return vs * max(1, int(round(target / float(vs))))

    # ------------------------------------------------------------------ global energy estimation -
    @staticmethod
    def _remaps_from_arrays(em, rm):
        eo = np.argsort(em, kind="stable")
        ro = np.argsort(rm, kind="stable")
        return em, rm, em[eo], eo, rm[ro], ro

    def _remaps(self, uid):
        """(ent_remap, rel_remap, sorted entity ids, their order, sorted relation ids, their order) of a
        universe; the sorted helpers are built on first use (the training commit and the LP fold read only the
        remaps, _remap_arrays)."""
        c = self._remap_cache.get(uid)
        if c is not None and len(c) == 2:
            c = self._remap_cache[uid] = self._remaps_from_arrays(*c)
        if c is None:
            emap, rmap = self.entity_id_mappings[uid], self.relation_id_mappings[uid]
            em = np.zeros(len(emap), dtype=np.int64)
            for g, l in emap.items():
                em[l] = g
            rm = np.zeros(len(rmap), dtype=np.int64)
            for g, l in rmap.items():
                rm[l] = g
            c = self._remap_cache[uid] = self._remaps_from_arrays(em, rm)
        return c

    def _remap_arrays(self, uid):
        """(local -> global entity ids, local -> global relation ids) of a universe."""
        c = self._remap_cache.get(uid)
        return (c[0], c[1]) if c is not None else self._remaps(uid)[:2]

    def _store(self, eval_mode):
        st = self._stores.get(eval_mode)
        if st is None:
            loader = self.data_loader if eval_mode == 'test' else self.valid_dataloader
            h, t, r = loader.eval_triples()
            dev = torch.device("cuda", torch.cuda.current_device())
            st = self._stores[eval_mode] = _KeyStore(h, t, r, self.ent_tot, dev)
        return st

    def _fold(self, st, universes):
        """MIN the scores of `universes` (this rank's trained ones) into the store's rows."""
        L = _native.lib()
        world, rank = _dist()
        local = [u for u in universes if u in self.trained_embedding_spaces]
        lp_us, pairs = [], []
        model_id = p_norm = norm_flag = None
        # the device local -> global entity maps of universes folded for the first time: one host-to-device copy
        # for all of them (views of one device array) instead of one per universe
        new = [u for u in local if u not in self._dev_remaps]
        if new:
            ems = [self._remap_arrays(u)[0] for u in new]
            flat = torch.from_numpy(np.concatenate(ems) if ems else np.zeros(0, np.int64)).cuda()
            off = 0
            for u, em in zip(new, ems):
                self._dev_remaps[u] = flat[off:off + len(em)]
                off += len(em)
        for slot, u in enumerate(local):
            kge = self.trained_embedding_spaces[u]
            if not next(kge.parameters()).is_cuda:
                kge.cuda()
            em, rm = self._remap_arrays(u)
            dr = self._dev_remaps[u]
            ent, rel, nv = kge.tables()
            U = _native.LpUniverse()
            U.ent, U.rel = ent.data_ptr(), rel.data_ptr()
            U.normv = nv.data_ptr() if nv is not None else None
            U.ent_total, U.rel_total, U.dim = ent.shape[0], rel.shape[0], ent.shape[1]
            U.d_ent_remap = dr.data_ptr()
            lp_us.append(U)
            model_id, p_norm, norm_flag = kge.native_model, int(kge.p_norm), 1 if kge.norm_flag else 0
            pairs.append((em, rm))
        pair_arr, arr_p = lp_pair_array([lp_pairs_all([p[0] for p in pairs], [p[1] for p in pairs], st.key_anchor,
                                                      st.key_rel, st.key_side)])
        if len(pair_arr):
            arr_u = (_native.LpUniverse * len(lp_us))(*lp_us)
            tup = st.tuple if self.missing_embedding_handling == 'null_vector' else None
            _native.check(L.pt_lp_min_scores(arr_u, len(lp_us), model_id, p_norm, norm_flag, arr_p, len(pair_arr),
                                             self.ent_tot, _native.ptr(st.rows), _native.ptr(tup), _native.stream()))
        min_combine([st.rows, st.tuple])

    def eval_universes(self, eval_mode):
        if self.incremental_strategy == "deprecate":
            raise NotImplementedError("the 'deprecate' incremental strategy is outside the accelerated path")
        st = self._store(eval_mode)
        start = self.current_tested_universes if eval_mode == 'test' else self.current_validated_universes
        start = max(start, 0)
        universes = list(range(start, self.next_universe_id))
        print("Global energy estimation.")
        print("- Mode: {}".format(eval_mode))
        if universes:
            print("- Universe range to obtain local energies: ({} -> {})".format(min(universes), max(universes)))
            self._fold(st, universes)
            st.folded = self.next_universe_id
            if eval_mode == 'test':
                self.current_tested_universes = self.next_universe_id
            elif eval_mode == 'valid':
                self.current_validated_universes = self.next_universe_id
        else:
            print("- No universes to be evaluated.")

    def _ranks(self, eval_mode, types=None):
        """raw / filtered ranks of every query of the split (head side, tail side) on the GPU; with `types`
        (Tester.device_type_lists) the type-constrained pair of each side follows."""
        L = _native.lib()
        st = self._store(eval_mode)
        known = L.pt_legacy_known()
        if not known:
            raise RuntimeError("no evaluation data imported (TestDataLoader.read() imports it)")
        dev = st.rows.device
        n = len(st.h)
        out = []
        r = np.ascontiguousarray(st.r, dtype=np.int64)
        for side, anchor, truth in ((0, st.t, st.h), (1, st.h, st.t)):
            # the split's queries, truths and known-partner lists do not change between validations: built
            # and uploaded once per (known set, side)
            ck = (int(known), side)
            if ck not in st.rank_inputs:
                off = np.zeros(n + 1, dtype=np.int64)
                a = np.ascontiguousarray(anchor, dtype=np.int64)
                _native.check(L.pt_known_partners(known, side, n, a.ctypes.data, r.ctypes.data, off.ctypes.data,
                                                  None))
                part = np.zeros(max(int(off[-1]), 1), dtype=np.int64)
                _native.check(L.pt_known_partners(known, side, n, a.ctypes.data, r.ctypes.data, off.ctypes.data,
                                                  part.ctypes.data))
                st.rank_inputs[ck] = (torch.from_numpy(st.q_row[side]).to(dev),
                                      torch.from_numpy(np.ascontiguousarray(truth, dtype=np.int64)).to(dev),
                                      torch.from_numpy(off).to(dev), torch.from_numpy(part).to(dev))
            d_row, d_truth, d_off, d_part = st.rank_inputs[ck]
            d_repl = st.tuple[d_row].contiguous() if self.missing_embedding_handling == 'null_vector' else None
            raw = torch.zeros(n, dtype=torch.int64, device=dev)
            filt = torch.zeros(n, dtype=torch.int64, device=dev)
            _native.check(L.pt_rank_rows(_native.ptr(st.rows), self.ent_tot, _native.ptr(d_row), _native.ptr(d_truth),
                                         _native.ptr(d_repl), _native.ptr(d_off), _native.ptr(d_part), n,
                                         _native.ptr(raw), _native.ptr(filt), _native.stream()))
            out.append((raw.cpu().numpy(), filt.cpu().numpy()))
            if types:
                d_rel = torch.from_numpy(r).to(dev)
                out.append(rank_types(L, st.rows, self.ent_tot, d_row, d_truth, d_repl, d_rel, types[side], d_off,
                                      d_part, n))
        if types:
            return [out[0], out[2], out[1], out[3]]   # head, tail, then the constrained head, tail
        return out   # [(raw_head, filt_head), (raw_tail, filt_tail)]

    def valid(self):
        """Filtered hit@10 of the validation split (validHead/validTail + getValidHit10, Valid.h:117-259)."""
        (_, fh), (_, ft) = self._ranks('valid')
        n = np.float32(max(len(fh), 1))
        lh = np.float32(np.count_nonzero(fh < 10)) / n
        rt = np.float32(np.count_nonzero(ft < 10)) / n
        return float((lh + rt) / np.float32(2))

    def global_energy_estimation(self, data):
        """Candidate-order score vector of one link-prediction query (:556-601), from the device rows."""
        mode = data['mode']
        batch_h, batch_t, batch_r = data['batch_h'], data['batch_t'], data['batch_r']
        rel = int(batch_r[0])
        if mode == 'head_batch':
            side, anchor, ents = 0, int(batch_t[0]), batch_h
        elif mode == 'tail_batch':
            side, anchor, ents = 1, int(batch_h[0]), batch_t
        else:
            raise ValueError("global_energy_estimation needs head_batch / tail_batch data")
        ents = np.asarray(ents, dtype=np.int64)
        scores = np.full(len(ents), np.inf, dtype=np.float32)
        repl = float("inf")
        for st in self._stores.values():
            k = st.row(side, anchor, rel)
            if k is not None and st.folded > 0:
                scores = st.rows[k].index_select(0, torch.from_numpy(ents).to(st.rows.device)).cpu().numpy()
                repl = float(st.tuple[k].item())
                break
        # scores MINed in by hand through obtain_embedding_space_score (the reference's dictionaries)
        key = get_string_key(anchor, rel)
        row = (self.evaluation_tail2head_triple_score_dict if side == 0
               else self.evaluation_head2tail_triple_score_dict).get(key)
        if row is not None:
            scores = np.minimum(scores, row[ents])
        t = (self.evaluation_tail2rel_tuple_score_dict if side == 0
             else self.evaluation_head2rel_tuple_score_dict).get(key)
        if t is not None and t < repl:
            repl = t
        if self.missing_embedding_handling == 'null_vector' and repl != float("inf"):
            scores[scores == np.inf] = repl
        return scores

    # ------------------------------------------- the reference's per-(key, universe) internals ----
    # eval_universes scores every (key, universe) pair of a split in two GPU launches into device key rows
    # (k_lp_bases / k_lp_scan). These are the reference's one-pair steps (:446-543), kept for callers that
    # drive them directly: the universe's scores come from one GPU predict, and the MIN goes into the
    # reference's score dictionaries (rows of entTotal floats, +inf default), which
    # global_energy_estimation reads together with the device rows.
    def _universe_key_scores(self, data, universe_id):
        """(global entity ids, scores) of every entity of universe `universe_id` as the missing side of
        data's key, in the universe's local id order (the reference's mapping order)."""
        mode = data['mode']
        mapping = self.entity_id_mappings[universe_id]
        rmap = self.relation_id_mappings[universe_id]
        sp = self.trained_embedding_spaces[universe_id]
        glob = np.fromiter(mapping.keys(), dtype=np.int64, count=len(mapping))
        loc = np.fromiter(mapping.values(), dtype=np.int64, count=len(mapping))
        anchor = [mapping[int(g)] for g in (data['batch_t'] if mode == 'head_batch' else data['batch_h'])]
        rel = [rmap[int(g)] for g in data['batch_r']]
        batch = {"batch_h": loc if mode == 'head_batch' else np.asarray(anchor, dtype=np.int64),
                 "batch_t": np.asarray(anchor, dtype=np.int64) if mode == 'head_batch' else loc,
                 "batch_r": np.asarray(rel, dtype=np.int64), "mode": mode}
        scores = np.asarray(sp.predict(batch), dtype=np.float32).reshape(-1)
        return glob, loc, scores

    def transmit_max_scores(self, data, embedding_space_mapping, scores):
        """:446-469: MIN a universe's scores (indexed by local id) into the key's global score row."""
        mode = data['mode']
        eval_rel_id = int(data['batch_r'][0])
        if mode == 'head_batch':
            eval_entity_id, score_dict = int(data['batch_t'][0]), self.evaluation_tail2head_triple_score_dict
        elif mode == 'tail_batch':
            eval_entity_id, score_dict = int(data['batch_h'][0]), self.evaluation_head2tail_triple_score_dict
        else:
            raise ValueError("transmit_max_scores needs head_batch / tail_batch data")
        row = score_dict.setdefault(get_string_key(eval_entity_id, eval_rel_id),
                                    np.full(self.ent_tot, np.inf, dtype=np.float32))
        glob = np.fromiter(embedding_space_mapping.keys(), dtype=np.int64, count=len(embedding_space_mapping))
        loc = np.fromiter(embedding_space_mapping.values(), dtype=np.int64, count=len(embedding_space_mapping))
        sc = np.asarray(scores.cpu().numpy() if isinstance(scores, torch.Tensor) else scores,
                        dtype=np.float32).reshape(-1)
        row[glob] = np.minimum(row[glob], sc[loc])

    def transmit_tuple_max_score(self, data, universe_id):
        """:494-512: MIN the universe's null-vector tuple score of the key into the tuple dictionary."""
        mode = data['mode']
        eval_rel_id = int(data['batch_r'][0])
        if mode == 'head_batch':
            eval_entity_id, score_dict = int(data['batch_t'][0]), self.evaluation_tail2rel_tuple_score_dict
        elif mode == 'tail_batch':
            eval_entity_id, score_dict = int(data['batch_h'][0]), self.evaluation_head2rel_tuple_score_dict
        else:
            raise ValueError("transmit_tuple_max_score needs head_batch / tail_batch data")
        key = get_string_key(eval_entity_id, eval_rel_id)
        sp = self.trained_embedding_spaces[universe_id]
        s = float(self.calc_tuple_score(self.entity_id_mappings[universe_id][eval_entity_id],
                                        self.relation_id_mappings[universe_id][eval_rel_id], mode,
                                        sp).reshape(-1)[0])
        if s < score_dict.get(key, float("inf")):
            score_dict[key] = s

    def obtain_embedding_space_score(self, data, universe_id):
        """:514-540: universe `universe_id`'s scores for data's key, MINed into the score dictionaries."""
        glob, loc, scores = self._universe_key_scores(data, universe_id)
        full = np.full(len(loc), np.inf, dtype=np.float32)
        full[loc] = scores
        self.transmit_max_scores(data, self.entity_id_mappings[universe_id], full)
        self.transmit_tuple_max_score(data, universe_id)

    def global_energy_estimation2(self, data):
        """:644-701: the key's candidate scores computed on the fly over the universes holding the anchor
        and the relation (no dictionaries), null-vector replacement included; scores in batch order."""
        mode = data['mode']
        bh, bt, br = (np.asarray(data[k].cpu().numpy() if isinstance(data[k], torch.Tensor) else data[k])
                      for k in ('batch_h', 'batch_t', 'batch_r'))
        anchor = int(bt[0] if mode == 'head_batch' else bh[0])
        rel = int(br[0])
        ents = np.asarray(bh if mode == 'head_batch' else bt, dtype=np.int64)
        row = np.full(self.ent_tot, np.inf, dtype=np.float32)
        tuple_score = float("inf")
        for u in self.gather_embedding_spaces(anchor, rel):
            if u not in self.trained_embedding_spaces:
                continue
            glob, loc, scores = self._universe_key_scores(
                {"batch_h": [anchor] if mode == 'tail_batch' else bh[:1], "batch_t": [anchor] if mode == 'head_batch'
                 else bt[:1], "batch_r": [rel], "mode": mode}, u)
            row[glob] = np.minimum(row[glob], scores)
            if self.missing_embedding_handling == 'null_vector':
                s = float(self.calc_tuple_score(self.entity_id_mappings[u][anchor], self.relation_id_mappings[u][rel],
                                                mode, self.trained_embedding_spaces[u]).reshape(-1)[0])
                tuple_score = s if s < tuple_score else tuple_score
        scores = row[ents]
        if self.missing_embedding_handling == 'null_vector' and tuple_score != float("inf"):
            scores[scores == np.inf] = tuple_score
        return scores

    def test_one_step(self, data):
        if data['mode'] in ('head_batch', 'tail_batch'):
            return self.global_energy_estimation(data)
        if data['mode'] != 'normal':
            raise ValueError("unknown evaluation mode %r" % (data['mode'],))
        # Parallel_Universe_Config.py:714-731. The reference unpacks `head, tail, rel = batch_h[i],
        # batch_r[i], batch_t[i]` and calls predict_triple(head, rel, tail): the triple it scores is
        # (h, relation = batch_t[i], tail = batch_r[i]). Kept as is (results identical to the reference).
        bh = np.asarray(data['batch_h'], dtype=np.int64)
        bt = np.asarray(data['batch_t'], dtype=np.int64)
        br = np.asarray(data['batch_r'], dtype=np.int64)
        heads, rels, tails = bh, bt, br
        score = self._predict_triples(heads, rels, tails)
        if self.missing_embedding_handling == "null_vector":
            for i in np.nonzero(score == np.inf)[0]:
                a = self.predict_tuple(int(heads[i]), int(rels[i]), mode="tail_batch")
                b = self.predict_tuple(int(tails[i]), int(rels[i]), mode="head_batch")
                score[i] = a if a < b else b
        return score

    def _predict_triples(self, heads, rels, tails):
        """predict_triple for many triples (Parallel_Universe_Config.py:413-442): min over the universes
        holding the head, the relation and the tail of that universe's score, +inf where none; one GPU
        predict launch per universe over all of its triples."""
        out = np.full(len(heads), np.inf, dtype=np.float32)
        per_u = defaultdict(list)
        for i in range(len(heads)):
            for u in self.gather_embedding_spaces(int(heads[i]), int(rels[i]), int(tails[i])):
                if u in self.trained_embedding_spaces:
                    per_u[u].append(i)
        for u in sorted(per_u):
            idx = np.asarray(per_u[u], dtype=np.int64)
            em, rm, eg, eo, rg, ro = self._remaps(u)
            sp = self.trained_embedding_spaces[u]
            s = sp.predict({"batch_h": lookup_local(eg, eo, heads[idx]), "batch_t": lookup_local(eg, eo, tails[idx]),
                            "batch_r": lookup_local(rg, ro, rels[idx]), "mode": "normal"})
            out[idx] = np.minimum(out[idx], np.asarray(s, dtype=np.float32).reshape(-1))
        return out

    def predict_tuple(self, ent_id, rel_id, mode):
        """Parallel_Universe_Config.py:390-411: min over the universes holding the entity and the relation
        of the null-vector tuple score."""
        best = float("inf")
        for u in self.gather_embedding_spaces(ent_id, rel_id):
            sp = self.trained_embedding_spaces.get(u)
            if sp is None:
                continue
            s = float(self.calc_tuple_score(self.entity_id_mappings[u][ent_id], self.relation_id_mappings[u][rel_id],
                                            mode, sp).reshape(-1)[0])
            best = s if s < best else best
        return best

    def run_link_prediction(self, type_constrain=False):
        self.data_loader.set_sampling_mode('link')
        self.eval_universes(eval_mode='test')
        L = _native.lib()
        types = device_type_lists(L, self._store('test').rows.device) if type_constrain else None
        ranks = self._ranks('test', types)
        (rh, fh), (rt, ft) = ranks[:2]
        met = np.zeros(10, dtype=np.float32)
        _native.check(L.pt_lp_metrics(rh.ctypes.data, fh.ctypes.data, rt.ctypes.data, ft.ctypes.data, len(rh),
                                      met.ctypes.data))
        self.last_ranks = (rh, fh, rt, ft)
        if type_constrain:   # the constrained metrics, as the reference's getters return them (Test.h:533-567)
            (crh, cfh), (crt, cft) = ranks[2:]
            self.last_tc_ranks = (crh, cfh, crt, cft)
            _native.check(L.pt_lp_metrics(crh.ctypes.data, cfh.ctypes.data, crt.ctypes.data, cft.ctypes.data,
                                          len(rh), met.ctypes.data))
        mrr, mr, hit10, hit3, hit1 = (float(x) for x in met[:5])
        print('Mean Reciprocal Rank: {}'.format(mrr))
        print('Mean Rank: {}'.format(mr))
        print('Hits@10: {}'.format(hit10))
        print('Hits@3: {}'.format(hit3))
        print('Hits@1: {}'.format(hit1))
        return mrr, mr, hit10, hit3, hit1

    def run_triple_classification(self, threshlod=None):
        # Parallel_Universe_Config.py:745-749 (the test split, negatives from getTestBatch)
        acc, threshlod = super().run_triple_classification(threshlod)
        print("Accuracy is: {}".format(acc))
        return acc, threshlod

    # file-driven triple classification (:751-818): labelled `h t r truth` files of a snapshot folder
    # `<in_path>/incremental/<snapshot>/`, scored by the same GPU predicts as the test split
    def tc_datastructure_adapter(self, pos_h, pos_t, pos_r, neg_h, neg_t, neg_r):
        """:753-765: one (positives, negatives) pair in the shape Tester.run_triple_classification iterates."""
        def arr(x):
            return np.asarray(x, dtype=np.int64) if len(x) else np.empty(0, dtype=np.int64)
        return [({'batch_h': arr(pos_h), 'batch_t': arr(pos_t), 'batch_r': arr(pos_r), "mode": "normal"},
                 {'batch_h': arr(neg_h), 'batch_t': arr(neg_t), 'batch_r': arr(neg_r), "mode": "normal"})]

    def load_triple_classification_file(self, file):
        """:767-789: `head tail rel truth_value` lines; truth 1 = positive, 0 = negative, others skipped."""
        pos, neg = ([], [], []), ([], [], [])
        with open(str(file), "rt", encoding="UTF-8") as f:
            for line in f:
                head, tail, rel, truth_value = line.split()
                dst = pos if truth_value == "1" else (neg if truth_value == "0" else None)
                if dst is not None:
                    dst[0].append(int(head))
                    dst[1].append(int(tail))
                    dst[2].append(int(rel))
        return pos[0], pos[1], pos[2], neg[0], neg[1], neg[2]

    def run_classification_of_deleted_triples(self, snapshot_idx, threshlod):
        """:791-800: accuracy at `threshlod` on every `tc_*` file of the snapshot folder."""
        folder = os.path.join(self.data_loader.in_path, "incremental", str(snapshot_idx))
        for name in sorted(os.listdir(folder)):
            if not name.startswith("tc_"):
                continue
            tc_data = self.tc_datastructure_adapter(*self.load_triple_classification_file(os.path.join(folder, name)))
            acc, _ = Tester.run_triple_classification(self, threshlod, data_iterator=tc_data)
            print("Accuracy for {} is: {}".format(name, acc))

    def run_triple_classification_from_files(self, snapshot):
        """:802-815: threshold and accuracy on the snapshot's prepared test examples, then the deleted-triple
        files at that threshold."""
        folder = os.path.join(self.data_loader.in_path, "incremental", str(snapshot))
        name = "triple_classification_prepared_test_examples.txt"
        tc_data = self.tc_datastructure_adapter(*self.load_triple_classification_file(os.path.join(folder, name)))
        acc, threshlod = Tester.run_triple_classification(self, data_iterator=tc_data)
        print("Accuracy for {} is: {}".format(name, acc))
        print("Determined threshold: {}".format(threshlod))
        print("Run negative triple classification...")
        self.run_classification_of_deleted_triples(snapshot, threshlod)
        return acc, threshlod

    def reset_evaluation_helpers(self):
        self.current_validated_universes = 0
        self.current_tested_universes = 0
        self._stores.clear()
        self.evaluation_head2tail_triple_score_dict.clear()
        self.evaluation_tail2head_triple_score_dict.clear()
        self.evaluation_head2rel_tuple_score_dict.clear()
        self.evaluation_tail2rel_tuple_score_dict.clear()
        self.incremental_strategy = "normal"

    # ------------------------------------------------------------------ single-triple helpers ---
    def gather_embedding_spaces(self, entity_1, rel, entity_2=None):
        ids = self.entity_universes[entity_1].intersection(self.relation_universes[rel])
        if entity_2 is not None:
            ids = ids.intersection(self.entity_universes[entity_2])
        return ids

    def calc_tuple_score(self, local_ent_id, local_rel_id, mode, embedding_space):
        dev = next(embedding_space.parameters()).device
        rel_embedding = embedding_space.rel_embeddings(torch.tensor([local_rel_id], device=dev).reshape(-1))
        ent = embedding_space.ent_embeddings(torch.tensor([local_ent_id], device=dev).reshape(-1))
        zero_vec = torch.tensor([[0.0]], device=dev)
        if mode == 'head_batch':
            return embedding_space._calc(zero_vec, ent, rel_embedding, mode)
        return embedding_space._calc(ent, zero_vec, rel_embedding, mode)

    def predict_triple(self, head_id, rel_id, tail_id, mode='normal'):
        best = float("inf")
        for u in self.gather_embedding_spaces(head_id, rel_id, tail_id):
            sp = self.trained_embedding_spaces.get(u)
            if sp is None:
                continue
            s = sp.predict({"batch_h": np.array([self.entity_id_mappings[u][head_id]]),
                            "batch_t": np.array([self.entity_id_mappings[u][tail_id]]),
                            "batch_r": np.array([self.relation_id_mappings[u][rel_id]]), "mode": mode})
            best = min(best, float(np.asarray(s).reshape(-1)[0]))
        return best

    # ------------------------------------------------------------------ state / checkpoints -----
    def save_model(self, filename=None, background=False):
        save_directory = self.checkpoint_dir
        if not filename:
            filename = "Pu{}_learned_spaces-{}_{}.ckpt".format(self.embedding_model.__name__,
                                                               self.next_universe_id, self.training_identifier)
        os.makedirs(save_directory, exist_ok=True)
        self.save_parameters(os.path.join("{}{}".format(save_directory, filename)), background=background)

    def save_best_state(self):
        self.best_state = self.get_state()

    def get_state(self):
        return {
            "trained_embedding_spaces": deepcopy(self.trained_embedding_spaces),
            "next_universe_id": self.next_universe_id,
            "entity_id_mappings": deepcopy(self.entity_id_mappings),
            "relation_id_mappings": deepcopy(self.relation_id_mappings),
            "entity_universes": deepcopy(self.entity_universes),
            "relation_universes": deepcopy(self.relation_universes),
        }

    def get_best_state(self):
        if self.best_state:
            print("Get best state...")
            self.trained_embedding_spaces = self.best_state["trained_embedding_spaces"]
            self.entity_id_mappings = self.best_state["entity_id_mappings"]
            self.relation_id_mappings = self.best_state["relation_id_mappings"]
            self.entity_universes = self.best_state["entity_universes"]
            self.relation_universes = self.best_state["relation_universes"]
            self.next_universe_id = self.best_state["next_universe_id"]
            self._remap_cache.clear()
            self._dev_remaps.clear()
        return self

    def extend_state_dict(self):
        return self._state_fields({k: getattr(self, k) for k in _MAP_KEYS})

    def _state_fields(self, maps):
        """extend_state_dict's layout (:890-899) with the four id-map entries taken from `maps`."""
        return {'initial_num_universes': self.initial_num_universes,
                'next_universe_id': self.next_universe_id,
                'trained_embedding_spaces': self.trained_embedding_spaces,
                'entity_id_mappings': maps['entity_id_mappings'],
                'relation_id_mappings': maps['relation_id_mappings'],
                'entity_universes': maps['entity_universes'],
                'relation_universes': maps['relation_universes'],
                'min_margin': self.min_margin,
                'max_margin': self.max_margin,
                'min_lr': self.min_lr,
                'max_lr': self.max_lr,
                'min_num_epochs': self.min_num_epochs,
                'max_num_epochs': self.max_num_epochs,
                'min_triple_constraint': self.min_triple_constraint,
                'max_triple_constraint': self.max_triple_constraint,
                'min_balance': self.min_balance,
                'max_balance': self.max_balance,
                'embedding_model': self.embedding_model,
                'embedding_model_param': self.embedding_model_param,
                'best_hit10': self.best_hit10,
                'bad_counts': self.bad_counts,
                'current_tested_universes': self.current_tested_universes,
                'current_validated_universes': self.current_validated_universes}

    def process_state_dict(self, state_dict):
        self.initial_num_universes = state_dict['initial_num_universes']
        self.next_universe_id = state_dict['next_universe_id']
        self.trained_embedding_spaces = state_dict['trained_embedding_spaces']
        self.entity_id_mappings = state_dict['entity_id_mappings']
        self.relation_id_mappings = state_dict['relation_id_mappings']
        self.entity_universes = state_dict['entity_universes']
        self.relation_universes = state_dict['relation_universes']
        self.min_margin = state_dict['min_margin']
        self.max_margin = state_dict['max_margin']
        self.min_lr = state_dict['min_lr']
        self.max_lr = state_dict['max_lr']
        self.min_num_epochs = state_dict['min_num_epochs']
        self.max_num_epochs = state_dict['max_num_epochs']
        self.min_triple_constraint = state_dict['min_triple_constraint']
        self.max_triple_constraint = state_dict['max_triple_constraint']
        if 'min_balance' in state_dict:
            self.min_balance = state_dict['min_balance']
            self.max_balance = state_dict['max_balance']
        elif 'embedding_model' in state_dict:   # the reference's elif (:906-912)
            self.embedding_model = state_dict['embedding_model']
            self.embedding_model_param = state_dict['embedding_model_param']
        if 'best_hit10' in state_dict:
            self.best_hit10 = state_dict['best_hit10']
            self.bad_counts = state_dict['bad_counts']
        # the reference never restores its score dictionaries (`if '' in state_dict`, :917): the next
        # evaluation re-folds every universe; the device rows start empty here for the same effect
        self._stores.clear()
        self.current_tested_universes = 0
        self.current_validated_universes = 0
        self._remap_cache.clear()
        self._dev_remaps.clear()

    def _gather_spaces(self):
        """Every rank's trained universes, assembled on rank 0 in id order as CPU modules (None on the
        other ranks): each rank sends (id, ent_tot, rel_tot, CPU state_dict) of the universes it holds with
        one gather_object; rank 0 rebuilds the modules with the model factory under a forked RNG (its
        torch stream is left untouched) and loads the gathered weights."""
        import torch.distributed as dist
        world, rank = _dist()
        mine = []
        for uid in sorted(self.trained_embedding_spaces):
            sp = self.trained_embedding_spaces[uid]
            mine.append((uid, int(sp.ent_tot), int(sp.rel_tot),
                         {k: v.detach().cpu() for k, v in sp.state_dict().items()}))
        got = [None] * world if rank == 0 else None
        dist.gather_object(mine, got, dst=0)
        if rank != 0:
            return None
        # a universe held by several ranks (the one-universe protocol, add_embedding_space, registers every
        # universe on every rank): the owner's copy, else the lowest rank's - after checking that every copy is
        # the same universe (sizes and table shapes equal), so a placement bug cannot pick a different universe.
        # Equal values are required only in the reference-order mode: the fast kernels sum gradient rows in arrival
        # order, so two ranks' trainings of one universe may differ in rounding
        chosen = {}
        diverged = []
        for r, part in enumerate(got):
            for x in part:
                uid = x[0]
                if uid in chosen:
                    y = chosen[uid][1]
                    same = (x[1], x[2]) == (y[1], y[2]) and x[3].keys() == y[3].keys() and all(
                        x[3][k].shape == y[3][k].shape for k in x[3])
                    if not same:
                        raise RuntimeError("universe %d is held by ranks %d and %d with different sizes"
                                           % (uid, chosen[uid][0], r))
                    if not all(torch.equal(x[3][k], y[3][k]) for k in x[3]):
                        if self.deterministic:
                            raise RuntimeError("universe %d is held by ranks %d and %d with different tables in the "
                                               "reference-order mode" % (uid, chosen[uid][0], r))
                        diverged.append(uid)
                if uid not in chosen or (chosen[uid][0] != self.owner(uid) and r == self.owner(uid)):
                    chosen[uid] = (r, x)
        if diverged:
            import warnings
            warnings.warn("universes %s: the ranks' copies differ in rounding (fast kernels); saving the owners' "
                          "copies" % sorted(set(diverged))[:8])
        spaces = defaultdict(Model)
        with torch.random.fork_rng(devices=[]):
            for uid in sorted(chosen):
                _, E_u, R_u, sd = chosen[uid][1]
                param = dict(self.embedding_model_param)
                if "dim" in param:   # the universe's own dim (a (lo, hi) dim range draws one per universe)
                    param["dim"] = int(sd["ent_embeddings.weight"].shape[1])
                m = self.embedding_model(E_u, R_u, **param)
                m.load_state_dict(sd)
                for p in m.parameters():
                    p.requires_grad = False
                spaces[uid] = m
        missing = [u for u in range(self.next_universe_id) if u not in spaces]
        if missing:
            raise RuntimeError("universes %s are held by no rank" % missing[:8])
        return spaces

    def _checkpoint_state(self):
        """extend_state_dict() as written: the id maps and occurrence sets pre-pickled (_Pickled) - straight
        from the registered remap arrays while the dictionaries hold nothing else (_map_log, _map_pickle), else
        from the dictionaries - and the universe dict shallow-copied: a snapshot of this moment (trained
        universes are not modified later)."""
        log = self.__dict__.get("_map_log")
        if log is not None and any(b[0] <= a[0] for a, b in zip(log, log[1:])):
            # a universe id registered twice (process_universe_mappings called again for one next_universe_id:
            # the reference merges the second call into the same dictionaries): the streams cannot express that
            log = self.__dict__["_map_log"] = None
        if log is not None and not self.__dict__.get("_maps_exposed"):
            uids = [x[0] for x in log]
            ems, rms = [x[1] for x in log], [x[2] for x in log]
            maps = {'entity_id_mappings': _Pickled(stream=_map_pickle.id_maps_stream(uids, ems)),
                    'relation_id_mappings': _Pickled(stream=_map_pickle.id_maps_stream(uids, rms)),
                    'entity_universes': _Pickled(stream=_map_pickle.universes_stream(uids, ems)),
                    'relation_universes': _Pickled(stream=_map_pickle.universes_stream(uids, rms))}
        else:
            maps = {k: _Pickled(getattr(self, k)) for k in _MAP_KEYS}
        state = dict(self._state_fields(maps))
        state['trained_embedding_spaces'] = copy(self.trained_embedding_spaces)
        return state

    def save_parameters(self, path, background=False):
        """One checkpoint file of the whole model, the reference's layout (:890-899). With several ranks
        every universe is gathered to rank 0, which alone writes; all ranks leave after the file exists.
        background=True (the training loop's best-model saves, one rank, static setting): the state is
        snapshotted here and the file written by a writer thread while training continues; the next save,
        load_parameters and the end of train_parallel_universes wait for it (flush_checkpoint). One rank writes
        through _checkpoint.UniverseArchive (the same file; each universe copied to the host and pickled once per
        run, the archive written by the library without the GIL)."""
        world, rank = _dist()
        if not (world == 1 and background and self.training_setting == "static"):
            self.flush_checkpoint()
        if world == 1:
            state = self._checkpoint_state()
            # universes already serialized by an earlier save are reused (_checkpoint.UniverseArchive)
            archive = self.__dict__.get("_ckpt_archive")
            if archive is None:
                archive = self._ckpt_archive = _checkpoint.UniverseArchive()
            if not (background and self.training_setting == "static"):
                _checkpoint.save(archive, state, path)
                return
            prev = getattr(self, "_ckpt_writer", None)
            err = prev[1] if prev is not None else []
            seq = self._ckpt_seq = getattr(self, "_ckpt_seq", 0) + 1
            latest = self.__dict__.setdefault("_ckpt_latest", {})
            latest[path] = seq
            writes = self.__dict__.setdefault("_ckpt_write_s", [])   # wall seconds of each background write

            def write():
                # writes land in save order: a writer first waits for the one before it (off the training thread)
                if prev is not None:
                    prev[0].join()
                if err:
                    return
                # a newer save of the same file was requested meanwhile: it writes the newer snapshot (the file only
                # skips an intermediate state it would have held until then)
                if latest.get(path) != seq:
                    return
                # written next to the target and renamed onto it: a crash or kill while the writer runs leaves the
                # previous checkpoint intact
                tmp = "%s.tmp%d" % (path, os.getpid())
                try:
                    t0 = time.perf_counter()
                    _checkpoint.save(archive, state, tmp, final_path=path)
                    os.replace(tmp, path)
                    writes.append(time.perf_counter() - t0)
                except BaseException as e:   # re-raised by flush_checkpoint on the caller's thread
                    err.append(e)
                    try:
                        os.remove(tmp)
                    except OSError:
                        pass
            # while a writer pickles (holding the GIL), the training thread's every return from a GIL-releasing
            # call (a ctypes launch, a torch op, a print) would wait up to the 5 ms switch interval for it: a short
            # interval until the writes are flushed
            if prev is None:
                self._switch_interval = sys.getswitchinterval()
                sys.setswitchinterval(min(self._switch_interval, 2e-4))
            th = threading.Thread(target=write, name="universe-checkpoint")
            th.start()
            self._ckpt_writer = (th, err)
            return
        import torch.distributed as dist
        spaces = self._gather_spaces()
        if rank == 0:
            state = self._checkpoint_state()
            state['trained_embedding_spaces'] = spaces
            torch.save(state, path, pickle_protocol=_checkpoint.PICKLE_PROTOCOL)
        dist.barrier()

    def flush_checkpoint(self):
        """Wait for a background checkpoint write (save_parameters(background=True)); re-raise its error."""
        w = getattr(self, "_ckpt_writer", None)
        if w is None:
            return
        self._ckpt_writer = None
        w[0].join()   # (the last writer joined its predecessors)
        sys.setswitchinterval(getattr(self, "_switch_interval", 0.005))
        if w[1]:
            raise w[1][0]

    def load_parameters(self, filename):
        """Load a save_parameters checkpoint (from any world size) and re-shard it over this job's ranks:
        the universes are placed by LPT on their evaluation cost (entities x dim) and each rank keeps
        only its own, moved to its GPU when there is one; the id maps stay complete on every rank."""
        self.flush_checkpoint()
        # checkpoints written by save_parameters (models + python containers): a full unpickle of a
        # file this code wrote
        state_dict = torch.load(self.checkpoint_dir + filename, weights_only=False, map_location="cpu")
        self.process_state_dict(state_dict)
        world, rank = _dist()
        spaces = self.trained_embedding_spaces
        self.universe_owners = {}
        if world > 1:
            self.universe_owners = place_universes(
                {uid: float(spaces[uid].ent_tot) * float(getattr(spaces[uid], "dim", 1)) for uid in spaces}, world)
            kept = defaultdict(Model)
            for uid in sorted(spaces):
                if self.universe_owners[uid] == rank:
                    kept[uid] = spaces[uid]
            self.trained_embedding_spaces = spaces = kept
        if torch.cuda.is_available():
            for sp in spaces.values():
                sp.cuda()

    def calculate_unembedded_ratio(self, mode='examine_entities'):
        num_unembedded = 0
        mapping_dict = self.entity_universes if mode == 'examine_entities' else self.relation_universes
        num_total = self.train_dataloader.entTotal if mode == 'examine_entities' else self.train_dataloader.relTotal
        for i in range(num_total):
            if len(mapping_dict[i]) == 0:
                num_unembedded += 1
        return num_unembedded / num_total

    def extend_parallel_universe(self, ParallelUniverse_inst):
        shift = self.next_universe_id
        for universe_id in list(ParallelUniverse_inst.trained_embedding_spaces.keys()):
            self.trained_embedding_spaces[universe_id + shift] = \
                ParallelUniverse_inst.trained_embedding_spaces[universe_id]
        for entity in range(ParallelUniverse_inst.ent_tot):
            self.entity_universes[entity].update(u + shift for u in ParallelUniverse_inst.entity_universes[entity])
        for relation in range(ParallelUniverse_inst.rel_tot):
            self.relation_universes[relation].update(
                u + shift for u in ParallelUniverse_inst.relation_universes[relation])
        for u in range(ParallelUniverse_inst.next_universe_id):
            for k, v in ParallelUniverse_inst.entity_id_mappings[u].items():
                self.entity_id_mappings[shift + u][k] = v
            for k, v in ParallelUniverse_inst.relation_id_mappings[u].items():
                self.relation_id_mappings[shift + u][k] = v
        self.next_universe_id += ParallelUniverse_inst.next_universe_id
