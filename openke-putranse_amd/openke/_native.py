"""ctypes binding of release/libputranse_hip.so (C-ABI declared in include/putranse.h).

The library is the only compute path: if it is missing, or no HIP device is visible, calls fail
loudly (NativeError / RuntimeError). There is no CPU fallback."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# The product library, in-tree. No environment variable selects another build: A/B measurements of two
# builds go through tools_gpu/ablib.py, which calls use_alternative_library() before anything loads it.
LIB_PATH = os.path.join(_HERE, "release", "libputranse_hip.so")
_LIB = None
_ALTERNATIVE = False

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_f32p = ctypes.POINTER(ctypes.c_float)

PT_TRANSE, PT_TRANSH = 0, 1
PT_SGD, PT_ADAGRAD = 0, 1
PT_DETERMINISTIC = 1   # pt_universes_train_ex flag: reference-order (deterministic) mode
# sampling paths of the counting-sort (large neg) step (include/putranse.h PT_PATH_*)
PT_PATH_TWO_PASS, PT_PATH_FUSED, PT_PATH_PART, PT_PATH_SAMPLED = 0, 1, 2, 3
PATH_KERNELS = {PT_PATH_TWO_PASS: ("k_sample_csr", "k_scan_counts"), PT_PATH_FUSED: ("k_sample_sort", "k_advance"),
                PT_PATH_PART: ("k_sample_part", None), PT_PATH_SAMPLED: (None, None)}


class NativeError(RuntimeError):
    pass


class ModelDesc(ctypes.Structure):
    _fields_ = [("model", c_i32), ("p_norm", c_i32), ("norm_flag", c_i32), ("opt", c_i32), ("lr", c_f32),
                ("margin", c_f32), ("ent_total", c_i64), ("rel_total", c_i64), ("dim", c_i64), ("ent", c_vp),
                ("rel", c_vp), ("normv", c_vp), ("ent_acc", c_vp), ("rel_acc", c_vp), ("norm_acc", c_vp)]


class UniverseJob(ctypes.Structure):
    _fields_ = [("graph", c_vp), ("seeds", c_vp), ("threads", c_i64), ("batch_size", c_i64), ("epochs", c_i64),
                ("nbatches", c_i64), ("neg", c_i64), ("lr", c_f32), ("margin", c_f32), ("ent", c_vp), ("rel", c_vp),
                ("normv", c_vp), ("ent_acc", c_vp), ("rel_acc", c_vp), ("norm_acc", c_vp), ("dim", c_i64)]


class TorchInitJob(ctypes.Structure):
    """pt_torch_init_job: initial tables of one model drawn on the GPU as torch's CPU generator draws them."""
    _fields_ = [("seed", ctypes.c_uint64), ("skip", c_i64), ("ntab", c_i32), ("pad_", c_i32),
                ("numel", c_i64 * 4), ("lo", ctypes.c_double * 4), ("hi", ctypes.c_double * 4), ("out", c_vp * 4)]


class LpUniverse(ctypes.Structure):
    _fields_ = [("ent", c_vp), ("rel", c_vp), ("normv", c_vp), ("ent_total", c_i64), ("rel_total", c_i64),
                ("dim", c_i64), ("d_ent_remap", c_vp)]


class ZipRecord(ctypes.Structure):
    """pt_zip_record: one stored record of a checkpoint archive."""
    _fields_ = [("name", ctypes.c_char_p), ("data", c_vp), ("size", c_i64), ("crc32", ctypes.c_uint32),
                ("crc_known", c_i32)]


class LpPair(ctypes.Structure):
    _fields_ = [("key", c_i32), ("universe", c_i32), ("anchor", c_i32), ("rel", c_i32), ("side", c_i32)]


# symbol -> (restype, argtypes); every symbol include/putranse.h declares
SIGNATURES = {
    "pt_last_error": (ctypes.c_char_p, []),
    "pt_version": (ctypes.c_int, []),
    "pt_graph_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(c_vp)]),
    "pt_graph_free": (ctypes.c_int, [c_vp]),
    "pt_set_count_header": (ctypes.c_int, [ctypes.c_int]),
    "pt_get_count_header": (ctypes.c_int, []),
    "pt_graph_ent_total": (c_i64, [c_vp]),
    "pt_graph_rel_total": (c_i64, [c_vp]),
    "pt_graph_train_total": (c_i64, [c_vp]),
    "pt_graph_triples": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
    "pt_sampler_create": (ctypes.c_int, [c_vp, c_i64, c_vp, ctypes.POINTER(c_vp)]),
    "pt_sampler_free": (ctypes.c_int, [c_vp]),
    "pt_sampler_set_seeds": (ctypes.c_int, [c_vp, c_vp]),
    "pt_sampler_get_seeds": (ctypes.c_int, [c_vp, c_vp]),
    "pt_sampler_sample": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "pt_sampler_sample_ex": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp,
                                            c_vp]),
    "pt_trainer_create": (ctypes.c_int, [ctypes.POINTER(ModelDesc), ctypes.POINTER(c_vp)]),
    "pt_trainer_free": (ctypes.c_int, [c_vp]),
    "pt_trainer_update_desc": (ctypes.c_int, [c_vp, ctypes.POINTER(ModelDesc)]),
    "pt_trainer_step": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "pt_trainer_run": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "pt_trainer_run_timed": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "pt_trainer_last_path": (ctypes.c_int, [c_vp]),
    "pt_trainer_set_deterministic": (ctypes.c_int, [c_vp, c_i32]),
    "pt_trainer_set_sampling": (ctypes.c_int, [c_vp, c_i32, c_i64]),
    "pt_trainer_set_sample_split": (ctypes.c_int, [c_vp, c_i64]),
    "pt_trainer_set_step_apply": (ctypes.c_int, [c_vp, c_i32]),
    "pt_universe_dim_supported": (ctypes.c_int, [c_i64, c_i32]),
    "pt_trainer_step_apply": (ctypes.c_int, [c_vp]),
    "pt_trainer_get_deterministic": (ctypes.c_int, [c_vp]),
    "pt_trainer_sample_csr": (ctypes.c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, ctypes.c_int32, c_vp,
                                             c_vp, c_vp, c_vp, c_vp]),
    "pt_score": (ctypes.c_int, [ctypes.POINTER(ModelDesc), c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "pt_score_queries": (ctypes.c_int, [ctypes.POINTER(ModelDesc), c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "pt_score_rows": (ctypes.c_int, [ctypes.POINTER(ModelDesc), c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "pt_lp_metrics": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "pt_universe_build": (ctypes.c_int, [c_vp, c_i64, c_i64, c_i64, c_f32, ctypes.POINTER(c_vp)]),
    "pt_universe_free": (ctypes.c_int, [c_vp]),
    "pt_universe_build_many": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    "pt_universe_ent_total": (c_i64, [c_vp]),
    "pt_universe_rel_total": (c_i64, [c_vp]),
    "pt_universe_train_total": (c_i64, [c_vp]),
    "pt_universe_remaps": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "pt_universe_graph": (c_vp, [c_vp]),
    "pt_universe_seeds": (ctypes.c_int, [c_vp, c_vp]),
    "pt_universe_set_create": (ctypes.c_int, [ctypes.POINTER(UniverseJob), c_i64, c_i32, c_i32, c_i32, c_i32,
                                              c_i64, c_i64, ctypes.POINTER(c_vp)]),
    "pt_universe_set_train": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "pt_universe_set_free": (ctypes.c_int, [c_vp]),
    "pt_universe_set_profile": (ctypes.c_int, [c_vp, c_vp]),
    "pt_universe_set_deterministic": (ctypes.c_int, [c_vp, c_i32]),
    "pt_universe_set_profiling": (ctypes.c_int, [c_vp, c_i32]),
    "pt_set_universe_team_width": (ctypes.c_int, [c_i32]),
    "pt_get_universe_team_width": (c_i32, []),
    "pt_universe_set_teams": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "pt_universe_set_states": (ctypes.c_int, [c_vp, c_i64, c_vp]),
    "pt_universe_set_reset": (ctypes.c_int, [c_vp]),
    "pt_universe_set_launch_times": (ctypes.c_int, [c_vp, ctypes.c_int64, c_vp, c_vp]),
    "pt_universes_train": (ctypes.c_int, [ctypes.POINTER(UniverseJob), c_i64, c_i32, c_i32, c_i32, c_i32, c_i64,
                                          c_i64, c_vp, c_vp]),
    "pt_trainer_set_slot_scale": (ctypes.c_int, [c_vp, c_i32]),
    "pt_trainer_slot_scale": (ctypes.c_int, [c_vp]),
    "pt_torch_init_tables": (ctypes.c_int, [ctypes.POINTER(TorchInitJob), c_i64, c_vp]),
    "pt_universes_train_ex": (ctypes.c_int, [ctypes.POINTER(UniverseJob), c_i64, c_i32, c_i32, c_i32, c_i32, c_i64,
                                             c_i64, c_i32, c_vp, c_vp]),
    "pt_lp_min_scores": (ctypes.c_int, [ctypes.POINTER(LpUniverse), c_i64, c_i32, c_i32, c_i32,
                                        ctypes.POINTER(LpPair), c_i64, c_i64, c_vp, c_vp, c_vp]),
    "pt_rank_rows": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    "pt_rank_types": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp,
                                     c_vp, c_vp]),
    "pt_known_partners": (ctypes.c_int, [c_vp, c_i32, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "pt_pickle_id_maps": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "pt_zip_write": (ctypes.c_int, [ctypes.c_char_p, c_vp, c_i64, c_i32, c_i32, c_i32]),
    "pt_lp_pairs": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "pt_pickle_universe_sets": (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "pt_known_create": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(c_vp)]),
    "pt_known_free": (ctypes.c_int, [c_vp]),
    "pt_rank_queries": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_i32, c_vp, c_vp, c_vp, c_i64]),
    "pt_legacy_sampler": (c_vp, []),
    "pt_legacy_import_status": (ctypes.c_int, []),
    "pt_legacy_bern": (c_i64, []),
    "pt_legacy_graph": (c_vp, []),
    "pt_legacy_eval_triples": (c_i64, [c_i32, c_vp, c_vp, c_vp]),
    "pt_legacy_known": (c_vp, []),
    "pt_legacy_types": (c_i64, [c_i32, c_vp, c_vp, c_vp]),
    # Base.so surface (argument types as the reference's loaders declare them)
    "setInPath": (None, [ctypes.c_char_p]),
    "setOutPath": (None, [ctypes.c_char_p]),
    "setWorkThreads": (None, [c_i64]),
    "getWorkThreads": (c_i64, []),
    "setBern": (None, [c_i64]),
    "setRandomSeed": (None, [c_i64]),
    "getRandomSeed": (c_i64, []),
    "randReset": (None, []),
    "importTrainFiles": (None, []),
    "getEntityTotal": (c_i64, []),
    "getRelationTotal": (c_i64, []),
    "getTrainTotal": (c_i64, []),
    "getTestTotal": (c_i64, []),
    "getValidTotal": (c_i64, []),
    "getTripleTotal": (c_i64, []),
    "sampling": (None, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64]),
    "getParallelUniverse": (None, [c_i64, c_f32]),
    "getEntityTotalUniverse": (c_i64, []),
    "getRelationTotalUniverse": (c_i64, []),
    "getTrainTotalUniverse": (c_i64, []),
    "getEntityRemapping": (None, [c_vp]),
    "getRelationRemapping": (None, [c_vp]),
    "swapHelpers": (None, []),
    "resetUniverse": (None, []),
    "activateLoadOfAllTriples": (None, [c_i64]),
    "importTestFiles": (None, []),
    "importTypeFiles": (None, []),
    "getNumOfNegatives": (c_i64, [c_i64, c_i64, c_i64]),
    "getNumOfPositives": (c_i64, [c_i64, c_i64, c_i64]),
    "getNegativeEntities": (None, [c_vp, c_i64, c_i64, c_i64]),
    "getPositiveEntities": (None, [c_vp, c_i64, c_i64, c_i64]),
    "getNumOfEntityRelations": (c_i64, [c_i64, c_i64]),
    "getEntityRelations": (None, [c_vp, c_i64, c_i64]),
    "initTest": (None, []),
    "getHeadBatch": (None, [c_vp, c_vp, c_vp]),
    "getTailBatch": (None, [c_vp, c_vp, c_vp]),
    "getTestBatch": (None, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "testHead": (None, [c_vp, c_i64, c_i64]),
    "testTail": (None, [c_vp, c_i64, c_i64]),
    "test_link_prediction": (None, [c_i64]),
    "getTestLinkMRR": (c_f32, [c_i64]),
    "getTestLinkMR": (c_f32, [c_i64]),
    "getTestLinkHit10": (c_f32, [c_i64]),
    "getTestLinkHit3": (c_f32, [c_i64]),
    "getTestLinkHit1": (c_f32, [c_i64]),
    "validInit": (None, []),
    "getValidHeadBatch": (None, [c_vp, c_vp, c_vp]),
    "getValidTailBatch": (None, [c_vp, c_vp, c_vp]),
    "validHead": (None, [c_vp, c_i64]),
    "validTail": (None, [c_vp, c_i64]),
    "getValidHit10": (c_f32, []),
}


def lib():
    """The loaded library (raises if it was not built: run `make -C openke-putranse_amd`)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError("libputranse_hip.so not built (%s); run __graft_entry__.build() or "
                              "make -C openke-putranse_amd" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if _ALTERNATIVE and not hasattr(L, name):
                continue   # an older build under A/B: entry points added since are absent
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def use_alternative_library(path):
    """Measurement tooling only (tools_gpu/ablib.py): load another build of the library instead of the
    product one. Must run before the first lib() call of the process."""
    global LIB_PATH, _ALTERNATIVE
    if _LIB is not None:
        raise NativeError("use_alternative_library: the library is already loaded (%s)" % LIB_PATH)
    LIB_PATH = os.path.abspath(path)
    _ALTERNATIVE = True


def check(rc):
    if rc != 0:
        raise NativeError(lib().pt_last_error().decode())


def require_gpu():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("openke (MI355X build) needs a visible HIP device: the hot path runs only in "
                           "libputranse_hip.so kernels and has no CPU fallback")


def stream():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
