"""Real-scale fixtures: the reference's own benchmark folders and trained tables, stored as data.

`tests/golden/real_<name>.npz` holds a benchmark folder of the reference (`benchmarks/WN18`, a slice of
`benchmarks/FB15K`) as integer arrays plus, verbatim, its `type_constrain.txt`. `write_dataset` turns it
back into the reference's headerless folder layout (`entity2id.txt` / `relation2id.txt` are only counted
by the reader, Reader.h:176-196, so they hold one line per id). `tests/golden/make_golden.py` runs the
reference on the folder this function writes, so the tests and the reference read the same bytes.
"""
import os

import numpy as np

SPLITS = ("train2id.txt", "valid2id.txt", "test2id.txt")


def read_triples(path, rows=None):
    a = np.loadtxt(path, dtype=np.int64, ndmin=2)
    return a if rows is None else a[rows[0]:rows[1]]


def pack_dataset(out_npz, ent_total, rel_total, splits, type_file=None, source=""):
    """splits: {file name: int array [n][3] (h t r)}."""
    arrs = {"ent_total": np.int64(ent_total), "rel_total": np.int64(rel_total), "source": np.str_(source)}
    for f in SPLITS:
        a = np.ascontiguousarray(splits[f], dtype=np.int64)
        small = np.uint16 if max(ent_total, rel_total) < 65536 else np.int32
        arrs[f.split(".")[0]] = a.astype(small)
    if type_file is not None:
        arrs["type_constrain"] = np.frombuffer(open(type_file, "rb").read(), dtype=np.uint8)
    np.savez_compressed(out_npz, **arrs)


def write_dataset(npz_path, out_dir):
    """Write the folder (idempotent); returns it with a trailing separator, as the loaders expect."""
    z = np.load(npz_path, allow_pickle=False)
    os.makedirs(out_dir, exist_ok=True)
    stamp = os.path.join(out_dir, ".complete")
    if not os.path.exists(stamp):
        E, R = int(z["ent_total"]), int(z["rel_total"])
        with open(os.path.join(out_dir, "entity2id.txt"), "w") as f:
            f.write("".join("e%d\t%d\n" % (i, i) for i in range(E)))
        with open(os.path.join(out_dir, "relation2id.txt"), "w") as f:
            f.write("".join("r%d\t%d\n" % (i, i) for i in range(R)))
        for name in SPLITS:
            a = z[name.split(".")[0]].astype(np.int64)
            with open(os.path.join(out_dir, name), "w") as f:
                f.write("".join("%d %d %d\n" % (h, t, r) for h, t, r in a))
        if "type_constrain" in z.files:
            with open(os.path.join(out_dir, "type_constrain.txt"), "wb") as f:
                f.write(z["type_constrain"].tobytes())
        open(stamp, "w").close()
    return os.path.join(out_dir, "")
