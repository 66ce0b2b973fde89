"""Synthetic knowledge-graph generator (benchmark and test inputs).

Writes a dataset directory in the reference's *headerless* format (one ``h t r``
triple per line; ``entity2id.txt`` / ``relation2id.txt`` are only line-counted),
which is what the reference reader expects (openke/base/Reader.h:176-196 counts
lines instead of reading a header).  The recipe follows SURVEY.md §8(d): numpy
``PCG64`` with a fixed seed, Zipf-like entity endpoints, a skewed relation
distribution, deduplicated triples.  No network, no real dataset needed.
"""
import os
import numpy as np

# name -> (entities, relations, train triples, valid, test)   shapes from SURVEY.md §8(a)
SHAPES = {
    "wn18":     (40943, 18, 141442, 5000, 5000),
    "fb15k237": (14541, 237, 272115, 17535, 20466),
    "wikidata": (35837, 121, 305631, 6000, 6000),
    "fb15k":    (14951, 1345, 483142, 50000, 59071),
    "small":    (500, 7, 3000, 100, 100),
    "tiny":     (60, 4, 300, 20, 20),
}
# Zipf exponent of the entity-endpoint distribution per shape (tuned so max/median degree
# land near the real dataset's: WN18 max 961 / median 4, FB15K237 max 7,614 / median 22).
ENT_SKEW = {"wn18": 0.5, "fb15k237": 0.7, "wikidata": 0.7, "fb15k": 0.7, "small": 0.6, "tiny": 0.5}


def _zipf_weights(n, a, rng):
    w = 1.0 / np.power(np.arange(1, n + 1, dtype=np.float64), a)
    rng.shuffle(w)
    return w / w.sum()


def generate(n_ent, n_rel, n_train, n_valid, n_test, seed=0, ent_skew=0.8, rel_skew=1.1):
    """Return (train, valid, test) int64 arrays of shape (n, 3) in (h, t, r) column order."""
    rng = np.random.Generator(np.random.PCG64(seed))
    pe = _zipf_weights(n_ent, ent_skew, rng)
    pr = _zipf_weights(n_rel, rel_skew, rng)
    pr = 0.5 * pr + 0.5 / n_rel          # every relation keeps a reasonable frequency floor
    need = n_train + n_valid + n_test
    keys = np.empty(0, dtype=np.int64)
    while keys.size < need:
        m = int((need - keys.size) * 1.3) + 1024
        h = rng.choice(n_ent, size=m, p=pe)
        t = rng.choice(n_ent, size=m, p=pe)
        r = rng.choice(n_rel, size=m, p=pr)
        ok = h != t
        k = (h[ok].astype(np.int64) * n_ent + t[ok]) * n_rel + r[ok]
        # keep first occurrence order while deduplicating
        allk = np.concatenate([keys, k])
        _, first = np.unique(allk, return_index=True)
        keys = allk[np.sort(first)]
    keys = keys[:need]
    perm = rng.permutation(need)
    keys = keys[perm]
    r = keys % n_rel
    ht = keys // n_rel
    t = ht % n_ent
    h = ht // n_ent
    trip = np.stack([h, t, r], axis=1).astype(np.int64)
    return trip[:n_train], trip[n_train:n_train + n_valid], trip[n_train + n_valid:]


def write_dataset(path, n_ent, n_rel, n_train, n_valid, n_test, seed=0, ent_skew=0.7):
    os.makedirs(path, exist_ok=True)
    train, valid, test = generate(n_ent, n_rel, n_train, n_valid, n_test, seed, ent_skew=ent_skew)
    with open(os.path.join(path, "entity2id.txt"), "w") as f:
        f.write("".join("e%d\t%d\n" % (i, i) for i in range(n_ent)))
    with open(os.path.join(path, "relation2id.txt"), "w") as f:
        f.write("".join("r%d\t%d\n" % (i, i) for i in range(n_rel)))
    for name, arr in (("train2id.txt", train), ("valid2id.txt", valid), ("test2id.txt", test)):
        np.savetxt(os.path.join(path, name), arr, fmt="%d")
    return path


def ensure_dataset(root, shape, seed=0):
    """Create (once) and return the directory of a named synthetic dataset shape."""
    path = os.path.join(root, "%s_s%d" % (shape, seed)) + os.sep
    if not os.path.exists(os.path.join(path, "test2id.txt")):
        write_dataset(path, *SHAPES[shape], seed=seed, ent_skew=ENT_SKEW[shape])
    return path


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("shape", choices=sorted(SHAPES))
    ap.add_argument("out")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    print(write_dataset(a.out, *SHAPES[a.shape], seed=a.seed, ent_skew=ENT_SKEW[a.shape]))
