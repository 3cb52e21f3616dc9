"""Deterministic synthetic inputs with the shapes of the reference's configs.

The real datasets (ogbn-arxiv, Reddit, products, ML-1M) are not available offline, so tests and
bench.py use statistics-matched stand-ins: a symmetric binary Chung–Lu power-law graph with the
config's node count and mean degree, N(0,1) features (the reference standardises features,
utils_graphsaint.py:40-43), and "logits" from a random linear map of the propagated features (the
reference's k-means input is a linear MLP's output, models/gcn.py:497-501). Everything is drawn
from numpy's PCG64 ``default_rng(seed)``, which is bit-identical across platforms.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp


@dataclass(frozen=True)
class Config:
    name: str
    n: int
    d: int
    n_classes: int
    avg_degree: float  # off-diagonal stored entries per row of the symmetric adjacency
    T: int
    alpha: float
    k: int
    kmeans: str  # "minibatch" | "lloyd"
    batch: int = 1000
    seed: int = 15


CONFIGS = {
    # Cora, reduction_rate 0.5 -> k = int(140 * 0.5)
    "cora": Config("cora", 2708, 1433, 7, 3.9, 5, 0.8, 70, "lloyd"),
    # config 2: ogbn-arxiv r=0.005 -> k = int(90941 * 0.005); nnz ~ 2.32M off-diagonal
    "arxiv": Config("ogbn-arxiv", 169343, 128, 40, 13.7, 18, 0.91, 454, "minibatch"),
    # config 3: Reddit inductive, train subgraph
    "reddit": Config("reddit", 153932, 602, 41, 66.0, 20, 0.95, 769, "minibatch"),
    # config 5: ogbn-products r=0.001 (T/alpha from arxiv; the reference gives none)
    "products": Config("ogbn-products", 2449029, 100, 47, 50.5, 18, 0.91, 196, "lloyd"),
}


def chung_lu(n: int, avg_degree: float, seed: int, gamma: float = 2.5) -> sp.csr_matrix:
    """Symmetric binary adjacency without self-loops, power-law expected degrees."""
    rng = np.random.default_rng(seed)
    w = (np.arange(1, n + 1, dtype=np.float64)) ** (-1.0 / (gamma - 1.0))
    rng.shuffle(w)
    p = w / w.sum()
    m = int(round(n * avg_degree / 2.0 * 1.04))  # head-room for duplicates/self-loops removed
    src = rng.choice(n, size=m, p=p)
    dst = rng.choice(n, size=m, p=p)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    rows = np.concatenate([src, dst]).astype(np.int64)
    cols = np.concatenate([dst, src]).astype(np.int64)
    A = sp.coo_matrix((np.ones(rows.shape[0], np.float32), (rows, cols)), shape=(n, n)).tocsr()
    A.sum_duplicates()
    A.data[:] = 1.0
    A.sort_indices()
    return A


def chung_lu_device(n: int, avg_degree: float, seed: int, device="cuda"):
    """:func:`chung_lu`'s model (weights rank^-1/1.5, symmetric, binary, no self-loops) sampled and
    canonicalised on the device with torch's generator — the host generator needs minutes at the
    ogbn-products shape. Not the same draws as :func:`chung_lu`. Returns a gdd CSRGraph."""
    import torch
    from .graph import CSRGraph
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    w = torch.arange(1, n + 1, device=device, dtype=torch.float64) ** (-1.0 / 1.5)
    w = w[torch.randperm(n, device=device, generator=g)].float()
    m = int(round(n * avg_degree / 2.0 * 1.04))
    src = torch.multinomial(w, m, replacement=True, generator=g)
    dst = torch.multinomial(w, m, replacement=True, generator=g)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    keys = torch.unique(torch.cat([src * n + dst, dst * n + src]))
    del src, dst, keep
    rows, col = keys // n, (keys % n).to(torch.int32)
    del keys
    rowptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    rowptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n), 0)
    return CSRGraph(rowptr.to(torch.int32), col, None, n)


def sbm_device(n: int, avg_degree: float, seed: int, block: int = 1024, p_in: float = 0.9,
               shuffle: bool = True, device="cuda", return_perm: bool = False):
    """A community-structured graph (stochastic block model: blocks of `block` consecutive nodes, a
    fraction p_in of each node's edges inside its block, the rest uniform), symmetric, binary, no
    self-loops, sampled on the device. With `shuffle` the node ids are permuted at random, as real
    graphs' ids carry no locality order. Returns a gdd CSRGraph (and, with `return_perm`, the id
    permutation: block member i is node perm[i]; None without `shuffle`)."""
    import torch
    from .graph import CSRGraph
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    m = int(round(n * avg_degree / 2.0 * 1.04))
    src = torch.randint(0, n, (m,), device=device, generator=g)
    inside = torch.rand(m, device=device, generator=g) < p_in
    b0 = (src // block) * block
    bsz = torch.clamp(n - b0, max=block)
    dst_in = b0 + (torch.rand(m, device=device, generator=g) * bsz).long().clamp(max=block - 1)
    dst = torch.where(inside, torch.minimum(dst_in, torch.full_like(dst_in, n - 1)),
                      torch.randint(0, n, (m,), device=device, generator=g))
    perm = None
    if shuffle:
        perm = torch.randperm(n, device=device, generator=g)
        src, dst = perm[src], perm[dst]
    keep = src != dst
    src, dst = src[keep], dst[keep]
    keys = torch.unique(torch.cat([src * n + dst, dst * n + src]))
    rows, col = keys // n, (keys % n).to(torch.int32)
    rowptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    rowptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n), 0)
    out = CSRGraph(rowptr.to(torch.int32), col, None, n)
    return (out, perm) if return_perm else out


def uniform_graph(n: int, avg_degree: float, seed: int) -> sp.csr_matrix:
    """Erdős–Rényi-style symmetric binary graph (worst-case gather locality variant)."""
    rng = np.random.default_rng(seed)
    m = int(round(n * avg_degree / 2.0))
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    keep = src != dst
    rows = np.concatenate([src[keep], dst[keep]])
    cols = np.concatenate([dst[keep], src[keep]])
    A = sp.coo_matrix((np.ones(rows.shape[0], np.float32), (rows, cols)), shape=(n, n)).tocsr()
    A.sum_duplicates()
    A.data[:] = 1.0
    A.sort_indices()
    return A


def features(n: int, d: int, seed: int) -> np.ndarray:
    return np.random.default_rng(seed + 1).standard_normal((n, d), dtype=np.float32)


def bag_of_words(n: int, d: int, seed: int, p: float = 0.0127) -> np.ndarray:
    """Cora-like row-normalised binary features."""
    rng = np.random.default_rng(seed + 2)
    x = (rng.random((n, d)) < p).astype(np.float32)
    x[np.arange(n), rng.integers(0, d, n)] = 1.0
    return x / x.sum(axis=1, keepdims=True)


def linear_logits(target: np.ndarray, n_classes: int, seed: int) -> np.ndarray:
    """A randomly initialised linear layer applied to the propagated features."""
    rng = np.random.default_rng(seed + 3)
    W = (rng.standard_normal((target.shape[1], n_classes)) / np.sqrt(target.shape[1])).astype(np.float32)
    b = (rng.standard_normal(n_classes) * 0.1).astype(np.float32)
    return target @ W + b


def blobs(n: int, dim: int, k: int, seed: int, spread: float = 3.0) -> np.ndarray:
    """Gaussian mixture around k random centres (k-means test input)."""
    rng = np.random.default_rng(seed)
    centres = rng.standard_normal((k, dim)) * spread
    lab = rng.integers(0, k, n)
    return (centres[lab] + rng.standard_normal((n, dim))).astype(np.float32)


def svd_like(n: int, dim: int, seed: int) -> np.ndarray:
    """Stand-in for distill_recsys.compute_svd_embeddings' U * sqrt(S) (distill_recsys.py:124-155):
    orthogonal-ish Gaussian columns scaled by the square root of a power-law singular spectrum, with
    a heavy-tailed per-row activity (popular users/items have larger embeddings)."""
    rng = np.random.default_rng(seed)
    s = np.sqrt(300.0 * np.arange(1, dim + 1, dtype=np.float64) ** -0.8)
    act = rng.pareto(2.5, n) + 0.2
    U = rng.standard_normal((n, dim)) / np.sqrt(n) * np.sqrt(act)[:, None] * 4.0
    return (U * s).astype(np.float32)
