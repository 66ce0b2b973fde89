"""Checkpoint engine of Parallel_Universe_Config.save_parameters (one rank; Parallel_Universe_Config.py:890-899).

The file is the one torch.save(state, path) writes - torch.load returns the same objects: the state dict, each
trained universe an nn.Module of its class with CPU tables - but a run's checkpoints are cumulative (every
best-model save holds every universe trained so far) and a trained universe never changes, so:

- each universe is serialized once: its tables copied device -> host together with the other universes new to
  the archive (one copy per segment, a storage of the archive shared by their tables), its module pickled once
  into a fragment of protocol-2 opcodes referring to that segment; a later checkpoint reuses the fragments and
  the segments (and the segments' CRC-32s) - only universes new since the last one are copied and pickled;
- data.pkl (pickle protocol 3) is assembled from fragments: the state dict's items pickled one by one (each fragment with its own
  memo, BINPUT before BINGET inside it) around the universes' fragments, with the tensors of the other entries
  (the pre-pickled id maps, _Pickled) as archive storages too;
- the archive is written by the library (pt_zip_write: torch's record layout and 64-byte data alignment, CRC-32s
  on several threads) with the GIL released, so a background write leaves the training thread running.

A state this cannot express (a table that is not float32, tables on several devices, one module object under two
universe ids) falls back to torch.save, and so does a run whose host copies would pass the archive's budget
(`max_host_bytes`: a quarter of the machine's memory, at most 16 GiB) - torch.save holds a checkpoint's copies only
while it writes."""
import ctypes
import io
import os
import pickle
import random
import sys
from collections import defaultdict

import torch
import torch.nn as nn

from .. import _native

_ALIGN = 64
# data.pkl's protocol: 3, not torch.save's default 2 - protocol 3 has BINBYTES (a bytes object in the state is
# copied as it is instead of through protocol 2's latin-1 text form) and, unlike 4, no frames (the fragments are
# concatenated). torch.load reads any protocol.
PICKLE_PROTOCOL = 3
_PROTO = bytes([0x80, PICKLE_PROTOCOL])


def _fragment_bytes(data):
    """A protocol-3 pickle without its PROTO header and STOP: an opcode fragment that pushes one object."""
    assert data[:2] == _PROTO and data[-1:] == b"."
    return data[2:-1]


class _Pickler(pickle.Pickler):
    """torch.save's persistent ids for storages, the keys handed out by the archive."""

    def __init__(self, f, archive):
        super().__init__(f, protocol=PICKLE_PROTOCOL)
        self._archive = archive

    def persistent_id(self, obj):
        if isinstance(obj, torch.storage.TypedStorage) or torch.is_storage(obj):
            return self._archive.storage_id(obj)
        return None


class _Unsupported(Exception):
    pass


def _signature(mod):
    """What a universe's cached fragment depends on: every parameter's and buffer's storage pointer, offset, shape,
    dtype, device and version counter, each parameter's requires_grad, and every submodule's training flag. A table
    replaced since the universe was serialized (`weight.data = ...`, `.to(...)`) or rewritten in place through
    autograd-visible ops (`add_` / `copy_` under no_grad, an optimizer step, load_state_dict) changes it. Writes
    through `.data` are invisible here as they are to autograd (torch gives `.data` its own version counter);
    `UniverseArchive.forget` drops a universe's fragment for callers that write that way."""
    mods = list(mod.modules())
    return (tuple((t.untyped_storage().data_ptr(), t.storage_offset(), tuple(t.shape), t.dtype, str(t.device),
                   t._version, bool(t.requires_grad)) for t in list(mod.parameters()) + list(mod.buffers())),
            tuple(m.training for m in mods))


def _shadow(mod, fills):
    """A module object like `mod` (same class, attributes, submodules) whose parameters / buffers are filled in
    later with host copies; `fills` collects (owner dict, name, source tensor, is_parameter)."""
    c = object.__new__(type(mod))
    c.__dict__.update(mod.__dict__)
    c._parameters = type(mod._parameters)(mod._parameters)
    c._buffers = type(mod._buffers)(mod._buffers)
    c._modules = type(mod._modules)((n, None if s is None else _shadow(s, fills)) for n, s in mod._modules.items())
    for name, p in mod._parameters.items():
        if p is not None:
            fills.append((c._parameters, name, p, True))
    for name, b in mod._buffers.items():
        if b is not None:
            fills.append((c._buffers, name, b, False))
    return c


class UniverseArchive(object):
    """Per-config cache of the universes' fragments and host segments (see the module docstring)."""

    def __init__(self, max_host_bytes=None):
        if max_host_bytes is None:
            try:
                phys = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
            except (ValueError, OSError, AttributeError):
                phys = 16 << 30
            max_host_bytes = min(16 << 30, phys // 4)
        self.max_host_bytes = int(max_host_bytes)
        self._frags = {}      # uid -> (module object, fragment bytes, segment key, table signature)
        self._segments = {}   # key -> [host uint8 tensor, crc32 or None]
        self._next_key = 0
        self._keys = {}       # storage _cdata -> key (segments and this write's other storages)
        self._storages = {}   # key -> storage, this write's non-segment storages
        self._used = set()
        self._stream = None

    # ---------------------------------------------------------------------------------- storages --
    def _new_key(self):
        k = str(self._next_key)
        self._next_key += 1
        return k

    def storage_id(self, obj):
        """torch.save's persistent id of a storage (torch/serialization.py _save.persistent_id)."""
        if isinstance(obj, torch.storage.TypedStorage):
            storage = obj._untyped_storage
            stype = getattr(torch, obj._pickle_storage_type())
            numel = obj._size()
        else:
            storage = obj
            stype = torch.serialization.normalize_storage_type(type(obj))
            numel = storage.nbytes()
        key = self._keys.get(storage._cdata)
        if key is None:
            key = self._keys[storage._cdata] = self._new_key()
            self._storages[key] = storage
        self._used.add(key)
        return ("storage", stype, key, torch.serialization.location_tag(storage), numel)

    def _pickle(self, obj):
        buf = io.BytesIO()
        _Pickler(buf, self).dump(obj)
        return _fragment_bytes(buf.getvalue())

    # --------------------------------------------------------------------------------- universes --
    def _add(self, items):
        """Fragments of the universes `items` [(uid, module)] over one new host segment."""
        fills, shadows = [], []
        for uid, m in items:
            f0 = len(fills)
            shadows.append((uid, m, _shadow(m, fills), f0))
        if any(t.dtype != torch.float32 for _, _, t, _ in fills):
            raise _Unsupported("non-float32 table")
        srcs = [t.detach() for _, _, t, _ in fills]
        devs = {t.device for t in srcs}
        if len(devs) > 1:
            raise _Unsupported("tables on several devices")
        numel = [t.numel() for t in srcs]
        total = sum(numel)
        held = sum(seg.numel() for seg, _ in self._segments.values())
        if held + 4 * total > self.max_host_bytes:
            raise _Unsupported("host copies over the archive's budget")
        dev = next(iter(devs)) if devs else torch.device("cpu")
        if dev.type == "cuda":
            if self._stream is None:
                self._stream = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(self._stream):   # the tables are final (their training launch was synchronised)
                flat = torch.cat([t.reshape(-1) for t in srcs]) if srcs else torch.zeros(0, device=dev)
                host = flat.cpu()
        else:   # numpy copies (torch's many small multi-threaded CPU copies are slow)
            host = torch.empty(total, dtype=torch.float32)
            hn = host.numpy()
            off = 0
            for t, n in zip(srcs, numel):
                hn[off:off + n] = t.reshape(-1).numpy()
                off += n
        seg = host.view(torch.uint8)
        key = self._new_key()
        self._segments[key] = [seg, None]
        self._keys[seg.untyped_storage()._cdata] = key
        off = 0
        for (owner, name, t, is_param), n in zip(fills, numel):
            v = host[off:off + n].view(t.shape)
            off += n
            if is_param:
                p = nn.Parameter(v, requires_grad=t.requires_grad)
                st = getattr(t, "__dict__", None)
                if st:
                    p.__dict__.update(st)
                owner[name] = p
            else:
                owner[name] = v
        before = set(self._storages)
        try:
            for uid, m, sh, _ in shadows:
                self._frags[uid] = (m, self._pickle(sh), key, _signature(m))
        finally:
            extra = [k for k in self._storages if k not in before]
            for k in extra:   # a storage outside the segment: write() would not hold it for the fragment
                self._keys.pop(self._storages.pop(k)._cdata, None)
        if extra:
            for uid, _, _, _ in shadows:
                self._frags.pop(uid, None)
            self._keys.pop(self._segments.pop(key)[0].untyped_storage()._cdata, None)
            raise _Unsupported("a universe module holds a tensor that is not a parameter or buffer")

    def forget(self, uid=None):
        """Drop the cached fragment of universe `uid` (all universes: None); its next save serializes it again."""
        if uid is None:
            self._frags.clear()
        else:
            self._frags.pop(uid, None)

    # ------------------------------------------------------------------------------------- write --
    def _data_pkl(self, state):
        out = [_PROTO, b"}("]
        for k, v in state.items():
            out.append(self._pickle(k))
            if k == "trained_embedding_spaces":
                empty = defaultdict(v.default_factory) if isinstance(v, defaultdict) else type(v)()
                out.append(self._pickle(empty))
                out.append(b"(")
                for uid in v:
                    out.append(self._pickle(uid))
                    out.append(self._frags[uid][1])
                out.append(b"u")
            else:
                out.append(self._pickle(v))
        out.append(b"u.")
        return b"".join(out)

    def write(self, path, state, threads=8, final_path=None, force_zip64=False):
        """torch.save(state, path), reusing what earlier writes of the same universes prepared; the archive's
        folder is named after final_path (the file `path` will be renamed to) as torch.save names it."""
        spaces = state.get("trained_embedding_spaces")
        if not isinstance(spaces, dict):
            raise _Unsupported("no universe dict")
        new = [(u, m) for u, m in spaces.items()
               if u not in self._frags or self._frags[u][0] is not m or self._frags[u][3] != _signature(m)]
        if len({id(m) for _, m in new}) != len(new) or any(not isinstance(m, nn.Module) for _, m in new):
            raise _Unsupported("universe objects")
        if new:
            self._add(new)
        self._storages, self._used = {}, set()
        try:
            data = self._data_pkl(state)
            for u in spaces:
                self._used.add(self._frags[u][2])
            records = []
            keep = [data]
            base = os.path.splitext(os.path.basename(final_path or path))[0] or "archive"

            def add(name, buf, n, crc=None):
                r = _native.ZipRecord()
                nb = ("%s/%s" % (base, name)).encode()
                keep.append(nb)
                r.name, r.data, r.size = nb, buf, n
                r.crc32, r.crc_known = (crc or 0), (1 if crc is not None else 0)
                records.append(r)

            def add_bytes(name, b):
                keep.append(b)
                add(name, ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) if b else None, len(b))

            add_bytes("data.pkl", data)
            add_bytes(".format_version", b"1")
            add_bytes(".storage_alignment", str(_ALIGN).encode())
            add_bytes("byteorder", sys.byteorder.encode())
            seg_rec = {}
            for key in sorted(self._used, key=int):
                if key in self._segments:
                    seg, crc = self._segments[key]
                    seg_rec[len(records)] = key
                    add("data/%s" % key, seg.data_ptr() if seg.numel() else None, seg.numel(), crc)
                else:
                    st = self._storages[key]
                    if st.device.type != "cpu":
                        st = st.cpu()
                    keep.append(st)
                    add("data/%s" % key, st.data_ptr() if st.nbytes() else None, st.nbytes())
            add_bytes("version", b"3\n")
            add_bytes(".data/serialization_id", ("%040d" % random.SystemRandom().randrange(10 ** 40)).encode())
            arr = (_native.ZipRecord * len(records))(*records)
            _native.check(_native.lib().pt_zip_write(path.encode(), arr, len(records), _ALIGN, threads,
                                                     1 if force_zip64 else 0))
            for i, key in seg_rec.items():
                self._segments[key][1] = arr[i].crc32
        finally:
            for k in list(self._storages):
                self._keys.pop(self._storages[k]._cdata, None)
            self._storages, self._used = {}, set()
        self._prune(spaces)

    def _prune(self, spaces):
        """Drop fragments of universes no longer held (a restored best state) and segments nothing uses."""
        for u in [u for u in self._frags if spaces.get(u) is not self._frags[u][0]]:
            del self._frags[u]   # (a re-serialized universe's entry was replaced by _add)
        live = {f[2] for f in self._frags.values()}
        for key in [k for k in self._segments if k not in live]:
            seg = self._segments.pop(key)[0]
            self._keys.pop(seg.untyped_storage()._cdata, None)


def save(archive, state, path, threads=8, final_path=None):
    """archive.write, or torch.save where the state holds something the archive does not express."""
    try:
        archive.write(path, state, threads, final_path)
    except _Unsupported:
        torch.save(state, path, pickle_protocol=PICKLE_PROTOCOL)
