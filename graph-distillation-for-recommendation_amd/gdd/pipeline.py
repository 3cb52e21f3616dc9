"""The reference's hot-path call sites as single functions (drop-ins for the agents and the recsys CLI).

* :func:`pretrained_clustering_hot_path` — the path of ``ClustGDD.pretrained_clustering``
  (clustgdd_agent_transduct.py:38-129): normalise the adjacency, propagate, cluster the caller's
  logits (MiniBatchKMeans for ogbn-arxiv, KMeans otherwise), per-cluster feature means and argmax
  labels. The MLP that produces the logits (models/gcn.py:626-653) is the caller's: pass the
  logits, or a callable that maps ``target_feat`` to them.
* :func:`kmeans_cluster` — ``distill_recsys.kmeans_cluster`` (distill_recsys.py:158-181):
  StandardScaler on the device (``gdd_standard_scaler``), then MiniBatchKMeans when
  ``minibatch and n > 20000`` else KMeans, ``n_init="auto"``; returns (labels int64, centres fp32).
* :func:`teacher_means` — the teacher super-node means (distill_recsys.py:623-636):
  ``index_add_`` sums over ``bincount(...).clamp_min(1)``, i.e. zero rows for empty clusters.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .cluster import argmax_rows, cluster_mean
from .graph import normalize_adj, propagate, to_csr
from .kmeans import KMeans, MiniBatchKMeans


def standard_scaler(X, device="cuda"):
    """StandardScaler().fit_transform(X) for fp32 X -> (X_scaled, mean_ fp64, scale_ fp64)."""
    lib = _lib.device_lib()
    Xd = (X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(X, np.float32)))
    Xd = Xd.to(device=device, dtype=torch.float32).contiguous()
    n, dim = Xd.shape
    out = torch.empty_like(Xd)
    mean = torch.empty(dim, dtype=torch.float64, device=Xd.device)
    scale = torch.empty(dim, dtype=torch.float64, device=Xd.device)
    _lib.check(lib.gdd_standard_scaler(n, dim, Xd.data_ptr(), out.data_ptr(), mean.data_ptr(),
                                       scale.data_ptr(), _lib.stream_ptr(Xd.device)))
    return out, mean, scale


def kmeans_cluster(X, n_clusters: int, seed: int, minibatch: bool = True, batch_size: int = 2048,
                   device="cuda"):
    """distill_recsys.kmeans_cluster on the device -> (labels int64 numpy, centres fp32 numpy)."""
    if n_clusters <= 0:
        raise ValueError("n_clusters must be > 0")
    n = X.shape[0]
    if n_clusters >= n:
        n_clusters = max(1, min(n_clusters, n))
    Xs, _, _ = standard_scaler(X, device=device)
    if minibatch and n > 20000:
        km = MiniBatchKMeans(n_clusters=n_clusters, random_state=seed, batch_size=batch_size,
                             n_init="auto", device=device)
    else:
        km = KMeans(n_clusters=n_clusters, random_state=seed, n_init="auto", device=device)
    km.fit(Xs)
    return km.labels_.astype(np.int64), km.cluster_centers_.astype(np.float32)


def teacher_means(emb: torch.Tensor, assignment, num_clusters: int) -> torch.Tensor:
    """index_add_ / bincount.clamp_min(1) super-node means (empty cluster -> zero row)."""
    out, _ = cluster_mean(emb.to(torch.float32), assignment, num_clusters, empty_as_zero=True)
    return out


def pretrained_clustering_hot_path(features, adj, T: int, alpha: float, logits, nnodes_syn: int,
                                   dataset: str = "", seed: int = 15, cluster_minibatch: int = 1000,
                                   device="cuda"):
    """The hot path of ClustGDD.pretrained_clustering.

    ``logits``: the MLP's embedding output (N x C), or a callable ``f(target_feat) -> logits``.
    Returns (cluster_feat_centers [k, d], cluster_center_labels int64 [k], cluster_labels int32 [N],
    adj_norm (CSRGraph), target_feat [N, d], prop_feat [N, d]) — the reference's outputs of this
    stage (transduct:129) without the MLP artefacts.
    """
    g = to_csr(adj, device=device)
    adj_norm = normalize_adj(g)                                  # transduct:46-50
    X = features if isinstance(features, torch.Tensor) else torch.from_numpy(
        np.ascontiguousarray(features, np.float32))
    X = X.to(device=device, dtype=torch.float32).contiguous()
    target_feat, prop_feat = propagate(adj_norm, X, T, alpha)  # transduct:59-65
    out = logits(target_feat) if callable(logits) else logits
    if dataset == "ogbn-arxiv":                                  # transduct:102-105
        km = MiniBatchKMeans(n_clusters=nnodes_syn, random_state=seed,
                             batch_size=cluster_minibatch, device=device).fit(out)
    else:
        km = KMeans(n_clusters=nnodes_syn, device=device).fit(out)
    feat_syn, _ = cluster_mean(target_feat, km.labels_device_, nnodes_syn)  # transduct:121-125
    labels_syn = argmax_rows(km.cluster_centers_device_)                    # transduct:126
    return feat_syn, labels_syn, km.labels_device_.to(torch.int32), adj_norm, target_feat, prop_feat
