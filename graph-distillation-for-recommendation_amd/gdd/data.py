"""Datasets for the ClustGDD drivers, with the attributes the agents read.

``utils.Transd2Ind`` (ClustGDD/utils.py:105-143) exposes a transductive dataset as: ``adj_full``,
``feat_full``, ``labels_full``, ``idx_train/val/test``, the role sub-graphs ``adj_train/val/test``
(``adj[np.ix_(idx, idx)]``), ``feat_*``, ``labels_*`` and ``nclass``. :class:`Transd2Ind` builds
the same object from arrays; :func:`synthetic` makes a learnable stand-in of a named dataset's
shape (the real Planetoid / OGB files cannot be downloaded here): class-conditioned Gaussian
features and a homophilous power-law graph, with the public split sizes (Cora: 20 train nodes
per class, 500 val, 1,000 test; ogbn-arxiv: OGB's 90,941 / 29,799 / 48,603; other shapes 54 / 18 / 28 %).
GraphSAINT-format directories load
through :func:`gdd.pipeline.load_graphsaint`.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

# name: (nodes, features, classes, mean degree, homophily)
SHAPES = {
    "cora": (2708, 1433, 7, 3.9, 0.81),
    "citeseer": (3327, 3703, 6, 2.7, 0.74),
    "pubmed": (19717, 500, 3, 4.5, 0.80),
    "ogbn-arxiv": (169343, 128, 40, 13.7, 0.65),
    "flickr": (89250, 500, 7, 10.1, 0.32),
    "reddit": (232965, 602, 41, 99.6, 0.78),
}


# public train / val / test sizes (ogbn-arxiv: OGB's time split; flickr / reddit: GraphSAINT's role.json)
SPLITS = {
    "ogbn-arxiv": (90941, 29799, 48603),
    "flickr": (44625, 22312, 22313),
    "reddit": (153932, 23699, 55334),
}


class Transd2Ind:
    """utils.Transd2Ind on arrays (keep_ratio 1): role sub-graphs and per-role features/labels."""

    def __init__(self, adj, features, labels, idx_train, idx_val, idx_test):
        adj = sp.csr_matrix(adj)
        labels = np.asarray(labels)
        self.nclass = int(labels.max()) + 1
        self.adj_full, self.feat_full, self.labels_full = adj, features, labels
        self.idx_train = np.array(idx_train)
        self.idx_val = np.array(idx_val)
        self.idx_test = np.array(idx_test)
        for role in ("train", "val", "test"):
            idx = getattr(self, "idx_" + role)
            setattr(self, "adj_" + role, adj[np.ix_(idx, idx)])
            setattr(self, "labels_" + role, labels[idx])
            setattr(self, "feat_" + role, features[idx])


def _graph(n, labels, avg_degree, homophily, rng):
    """Symmetric binary power-law graph; a fraction `homophily` of the edges stays inside a class."""
    w = np.arange(1, n + 1, dtype=np.float64) ** (-1.0 / 1.5)
    rng.shuffle(w)
    m = int(round(n * avg_degree / 2.0 * 1.05))
    p = w / w.sum()
    src = rng.choice(n, size=m, p=p)
    nclass = int(labels.max()) + 1
    members = [np.nonzero(labels == c)[0] for c in range(nclass)]
    probs = [w[idx] / w[idx].sum() for idx in members]
    same = rng.random(m) < homophily
    dst = rng.choice(n, size=m, p=p)
    for c in range(nclass):
        sel = np.nonzero(same & (labels[src] == c))[0]
        if sel.size:
            dst[sel] = rng.choice(members[c], size=sel.size, p=probs[c])
    keep = src != dst
    rows = np.concatenate([src[keep], dst[keep]])
    cols = np.concatenate([dst[keep], src[keep]])
    A = sp.coo_matrix((np.ones(rows.shape[0], np.float32), (rows, cols)), shape=(n, n)).tocsr()
    A.sum_duplicates()
    A.data[:] = 1.0
    A.sort_indices()
    return A


def synthetic(name: str, seed: int = 15, n: int | None = None, d: int | None = None,
              signal: float = 1.0) -> Transd2Ind:
    """A learnable dataset with `name`'s shape (SHAPES) and public split proportions."""
    n0, d0, nclass, deg, hom = SHAPES[name]
    n = n or n0
    d = d or d0
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, nclass, n)
    mu = rng.standard_normal((nclass, d)).astype(np.float32) * (signal / np.sqrt(max(d, 1)) * 4.0)
    feat = (mu[labels] + rng.standard_normal((n, d)).astype(np.float32)).astype(np.float32)
    A = _graph(n, labels, deg, hom, rng)
    if name in ("cora", "citeseer", "pubmed"):
        order = rng.permutation(n)
        idx_train = np.sort(np.concatenate([order[labels[order] == c][:20] for c in range(nclass)]))
        rest = np.setdiff1d(order, idx_train, assume_unique=False)
        rest = rest[rng.permutation(rest.shape[0])]
        idx_val, idx_test = np.sort(rest[:500]), np.sort(rest[500:1500])
    elif name in SPLITS and n == n0:  # the public split sizes (train, val, test)
        a, b = SPLITS[name][0], SPLITS[name][0] + SPLITS[name][1]
        idx_train, idx_val, idx_test = np.arange(a), np.arange(a, b), np.arange(b, n)
    else:
        a, b = int(0.54 * n), int(0.72 * n)
        idx_train, idx_val, idx_test = np.arange(a), np.arange(a, b), np.arange(b, n)
    return Transd2Ind(A, feat, labels, idx_train, idx_val, idx_test)
