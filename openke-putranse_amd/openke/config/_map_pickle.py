"""Pickle streams of the universe id maps (Parallel_Universe_Config.entity_id_mappings / relation_id_mappings /
entity_universes / relation_universes, the reference's dictionaries, Parallel_Universe_Config.py:90-95, 179-207)
written straight from the per-universe remap arrays, for the checkpoint (save_parameters): the same objects
pickle.loads gives back as for the materialised dictionaries - the same container types and default factories,
keys in the same insertion order, the same values and set members - without building the dictionaries first.

A stream uses only protocol-2/4 opcodes with explicit memo slots: GLOBAL ('c') for the container types, BINPUT /
BINGET, TUPLE1 + REDUCE for each defaultdict, MARK ... SETITEMS for dict items, EMPTY_SET + MARK ... ADDITEMS for
sets, and every integer as BININT (a 4-byte signed value: ids and universe numbers are < 2**31). The item
regions come from the library in one pass (pt_pickle_id_maps / pt_pickle_universe_sets, csrc/pickle_maps.cpp);
this module adds the container headers."""
import ctypes

import numpy as np

from .. import _native

_PROTO = b"\x80\x04"
_STOP = b"."
# the module holding defaultdict_int (the inner factory of the id maps): the reference's module path
_FACTORY_MODULE = b"openke.config.Parallel_Universe_Config"


def _items(fn, uids, remaps):
    L = _native.lib()
    n = len(uids)
    u = np.ascontiguousarray(uids, dtype=np.int64)
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum([len(r) for r in remaps], out=off[1:])
    ids = np.ascontiguousarray(np.concatenate(remaps) if n else np.zeros(0), dtype=np.int64)
    need = np.zeros(1, dtype=np.int64)
    _native.check(getattr(L, fn)(n, u.ctypes.data, off.ctypes.data, ids.ctypes.data, None, 0, need.ctypes.data))
    out = bytearray(int(need[0]))
    buf = (ctypes.c_uint8 * len(out)).from_buffer(out) if len(out) else None
    _native.check(getattr(L, fn)(n, u.ctypes.data, off.ctypes.data, ids.ctypes.data, buf, len(out),
                                 need.ctypes.data))
    return out


def id_maps_stream(uids, remaps):
    """defaultdict(defaultdict_int) {uids[u]: defaultdict(int){remaps[u][i]: i}} (entity_id_mappings /
    relation_id_mappings), universes in the given (ascending) order."""
    head = (_PROTO + b"ccollections\ndefaultdict\nq\x00cbuiltins\nint\nq\x010"
            + b"h\x00c" + _FACTORY_MODULE + b"\ndefaultdict_int\n\x85R")
    return bytes(head + b"(" + _items("pt_pickle_id_maps", uids, remaps) + b"u" + _STOP)


def universes_stream(uids, remaps):
    """defaultdict(set) id -> {universes holding it} (entity_universes / relation_universes) over universes
    `uids` (ascending) with local -> global id arrays `remaps`: keys in order of first appearance (universe by
    universe, local id order within one, as process_universe_mappings adds them), sets filled in universe order."""
    head = _PROTO + b"ccollections\ndefaultdict\ncbuiltins\nset\n\x85R"
    return bytes(head + b"(" + _items("pt_pickle_universe_sets", uids, remaps) + b"u" + _STOP)
