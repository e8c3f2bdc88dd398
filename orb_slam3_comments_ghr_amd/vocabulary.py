"""DBoW2 vocabulary (``TemplatedVocabulary<FORB::TDescriptor, FORB>``, ref:Thirdparty/DBoW2/DBoW2/
TemplatedVocabulary.h) on the GPU: ``ORBVocabulary.transform`` mirrors ``transform(features,
BowVector&, FeatureVector&, levelsup)`` as ``Frame::ComputeBoW`` calls it (ref:src/Frame.cc:995-1010).

``Vocabulary`` holds the reference's in-memory form (node 0 the root, nodes in file order with parent,
leaf flag, descriptor and weight; ref:TemplatedVocabulary.h:1334-1415) and reads / writes the text
format (ORBvoc.txt).  ORBvoc.txt itself is not in the container: ``synth_vocabulary`` builds trees of
the same shape (k-ary, L levels, TF-IDF weights) from seeded random descriptors.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import Context, _abi

TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)


def _p(a):
    return None if a is None else int(a.ctypes.data)


@dataclass
class Vocabulary:
    k: int
    L: int
    scoring: int
    weighting: int
    parent: np.ndarray     # n_nodes int32 (parent[0] unused)
    is_leaf: np.ndarray    # n_nodes uint8
    desc: np.ndarray       # n_nodes x 32 uint8
    weight: np.ndarray     # n_nodes float64

    def __post_init__(self):
        self.parent = np.ascontiguousarray(self.parent, np.int32)
        self.is_leaf = np.ascontiguousarray(self.is_leaf, np.uint8)
        self.desc = np.ascontiguousarray(self.desc, np.uint8).reshape(-1, 32)
        self.weight = np.ascontiguousarray(self.weight, np.float64)

    @property
    def n_nodes(self):
        return len(self.parent)

    @property
    def n_words(self):
        return int(self.is_leaf[1:].sum())

    def struct(self):
        s = _abi.OsgVocabularyDesc()
        s.k, s.L, s.scoring, s.weighting, s.n_nodes = self.k, self.L, self.scoring, self.weighting, self.n_nodes
        s.parent, s.is_leaf, s.desc, s.weight = _p(self.parent), _p(self.is_leaf), _p(self.desc), _p(self.weight)
        return s

    def to_text(self, path):
        """saveToTextFile's format (ref:TemplatedVocabulary.h:1468-1500): header, then one node per line."""
        with open(path, "w") as f:
            f.write(f"{self.k} {self.L}  {self.scoring} {self.weighting}\n")
            for i in range(1, self.n_nodes):
                d = " ".join(str(int(v)) for v in self.desc[i])
                f.write(f"{int(self.parent[i])} {int(self.is_leaf[i])} {d} {float(self.weight[i])!r}\n")

    @staticmethod
    def from_text(path) -> "Vocabulary":
        with open(path) as f:
            k, L, sc, wt = (int(x) for x in f.readline().split())
            parent, leaf, desc, weight = [0], [0], [np.zeros(32, np.uint8)], [0.0]
            for line in f:
                t = line.split()
                if not t:
                    continue
                parent.append(int(t[0]))
                leaf.append(1 if int(t[1]) > 0 else 0)
                desc.append(np.array([int(v) for v in t[2:34]], np.uint8))
                weight.append(float(t[34]))
        return Vocabulary(k, L, sc, wt, np.array(parent), np.array(leaf), np.stack(desc), np.array(weight))


def _flip(rng, rows, p):
    bits = np.unpackbits(rows, axis=1)
    return np.packbits(bits ^ (rng.random(bits.shape) < p).astype(np.uint8), axis=1)


def synth_vocabulary(rng, k=10, L=4, scoring=L1_NORM, weighting=TF_IDF, min_children=2, early_leaf=0.0,
                     min_leaf_depth=3, stop_frac=0.0, flip=(0.25, 0.18, 0.12, 0.08, 0.05, 0.03)):
    """A k-ary tree of L levels written in breadth-first file order (as saveToTextFile does).  Each
    internal node has U{min_children..k} children whose descriptors are noisy copies of the parent's
    (bit-flip probability shrinking with depth); with probability ``early_leaf`` a node deeper than
    ``min_leaf_depth`` - 1 becomes a leaf early.  Leaf weights are idf-like U(0.5, 8); a
    ``stop_frac`` of leaves get weight 0 (stopped words)."""
    parent, leaf, desc, depth = [0], [0], [rng.integers(0, 256, 32, dtype=np.uint8)], [0]
    frontier = [0]
    while frontier:
        nxt = []
        for p in frontier:
            nc = int(rng.integers(min_children, k + 1))
            d = depth[p] + 1
            kids = _flip(rng, np.repeat(desc[p][None], nc, 0), flip[min(d - 1, len(flip) - 1)])
            for c in range(nc):
                i = len(parent)
                parent.append(p)
                desc.append(kids[c])
                depth.append(d)
                is_leaf = d >= L or (d >= min_leaf_depth and rng.random() < early_leaf)
                leaf.append(1 if is_leaf else 0)
                if not is_leaf:
                    nxt.append(i)
        frontier = nxt
    n = len(parent)
    weight = np.where(np.array(leaf) == 1, rng.uniform(0.5, 8.0, n), 0.0)
    if stop_frac > 0:
        weight[(np.array(leaf) == 1) & (rng.random(n) < stop_frac)] = 0.0
    if weighting in (TF, BINARY):
        weight = np.where(weight > 0, 1.0, 0.0)
    weight[0] = 0.0
    desc = np.stack(desc)
    desc[0] = 0  # the root's descriptor is never compared (and not stored in the text format)
    return Vocabulary(k, L, scoring, weighting, np.array(parent), np.array(leaf), desc, weight)


def synth_features(rng, voc: Vocabulary, n=1200, flip=0.08, random_frac=0.2):
    """Descriptors near random leaves of the vocabulary (noisy copies), plus a fraction of uniform ones."""
    leaves = np.nonzero(voc.is_leaf)[0]
    src = voc.desc[rng.choice(leaves, n)]
    f = _flip(rng, src, flip)
    r = rng.random(n) < random_frac
    f[r] = rng.integers(0, 256, (int(r.sum()), 32), dtype=np.uint8)
    return f


@dataclass
class BowResult:
    """BowVector (ascending word ids, values) and FeatureVector (CSR: node ids ascending, each node's
    feature indices in feature order): the arrays osg_bow_side.fv takes."""
    word: np.ndarray
    value: np.ndarray
    node_id: np.ndarray
    node_start: np.ndarray
    feat: np.ndarray


def make_bow_out(n):
    o = _abi.OsgBowOut()
    bufs = (np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1), np.float64), np.zeros(max(n, 1), np.uint32),
            np.zeros(n + 1, np.int32), np.zeros(max(n, 1), np.int32))
    o.word, o.value, o.node_id, o.node_start, o.feat = (_p(b) for b in bufs)
    return o, bufs


def bow_result(o, bufs):
    w, v, nid, ns, ft = bufs
    nn = o.n_nodes
    m = int(ns[nn]) if nn else 0
    return BowResult(w[:o.n_words].copy(), v[:o.n_words].copy(), nid[:nn].copy(), ns[:nn + 1].copy(), ft[:m].copy())


class ORBVocabulary:
    """``ORBVocabulary`` (= TemplatedVocabulary<FORB::TDescriptor, FORB>) resident on the device."""

    def __init__(self, ctx: Context, voc: Vocabulary | None = None, text_path: str | None = None):
        self.ctx = ctx
        h = C.c_void_p()
        if text_path is not None:
            rc = ctx.lib.osg_vocabulary_load_text(ctx.handle, text_path.encode(), C.byref(h))
        else:
            s = voc.struct()
            rc = ctx.lib.osg_vocabulary_create(ctx.handle, C.byref(s), C.byref(h))
        ctx.check(rc, "vocabulary upload")
        self.handle = h

    def info(self):
        out = np.zeros(4, np.int32)
        self.ctx.lib.osg_vocabulary_info(self.handle, _p(out))
        return dict(k=int(out[0]), L=int(out[1]), n_nodes=int(out[2]), n_words=int(out[3]))

    def transform(self, desc: np.ndarray, levelsup: int = 4) -> BowResult:
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = desc.shape[0]
        o, bufs = make_bow_out(n)
        rc = self.ctx.lib.osg_vocabulary_transform(self.ctx.handle, self.handle, _p(desc), n, int(levelsup), C.byref(o))
        self.ctx.check(rc, "vocabulary transform")
        return bow_result(o, bufs)

    def transform_batch(self, descs, levelsup: int = 4) -> list:
        descs = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in descs]
        B = len(descs)
        ns = np.array([d.shape[0] for d in descs], np.int32)
        allv = np.concatenate(descs) if B else np.zeros((0, 32), np.uint8)
        outs = [make_bow_out(int(x)) for x in ns]
        arr = (_abi.OsgBowOut * max(B, 1))(*[o for o, _ in outs])
        rc = self.ctx.lib.osg_vocabulary_transform_batch(self.ctx.handle, self.handle, _p(allv), _p(ns), B,
                                                         int(levelsup), C.addressof(arr))
        self.ctx.check(rc, "vocabulary transform batch")
        return [bow_result(arr[i], outs[i][1]) for i in range(B)]

    def close(self):
        if self.handle:
            self.ctx.lib.osg_vocabulary_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
