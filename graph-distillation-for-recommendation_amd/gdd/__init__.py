"""gdd — MI355X-native hot path of ClustGDD graph distillation.

Drop-in replacements for the reference's hot-path call sites (see include/gdd.h for the C ABI and
the reference file:line each entry point replaces):

* :func:`gdd.graph.to_csr`, :func:`gdd.graph.normalize_adj_tensor`, :func:`gdd.graph.propagate`
* :class:`gdd.kmeans.KMeans`, :class:`gdd.kmeans.MiniBatchKMeans`
* :func:`gdd.cluster.cluster_mean`, :func:`gdd.cluster.argmax_rows`
* :mod:`gdd.pipeline` — ``pretrained_clustering_hot_path`` (the ClustGDD stage end to end),
  ``kmeans_cluster`` / ``teacher_means`` / ``standard_scaler`` (distill_recsys)
* :mod:`gdd.condense` — ``graph_sparse`` / ``graph_compress`` / ``ER_estimator`` /
  ``attaw_ER_estimator`` (ClustGDD's sparsification and cluster-level graph)
* :class:`gdd.sharded.ShardedKMeans` — Lloyd on several ranks: the E-step partitioned by rows, the
  M-step by clusters, all-gathers of the labels and the cluster slices (bit-identical to one GPU)
* :mod:`gdd.agent` / :mod:`gdd.agent_induct` — the transductive and inductive ClustGDD agents;
  :mod:`gdd.train_clustgdd_transduct` / :mod:`gdd.train_clustgdd_induct` /
  :mod:`gdd.distill_recsys` — the drop-in command lines
"""
from . import _lib  # noqa: F401  (imports torch first, see _lib docstring)
from . import gcn, pipeline, recsys  # noqa: F401
from .cluster import argmax_rows, cluster_mean, group_by_label
from .condense import ER_estimator, attaw_ER_estimator, graph_compress, graph_sparse
from .graph import (CSRGraph, induced_subgraph, normalize_adj, normalize_adj_tensor, propagate, spmm,
                    to_csr)
from .kmeans import KMeans, MiniBatchKMeans
from .sharded import ShardedKMeans, shard_rows

__all__ = [
    "CSRGraph", "to_csr", "normalize_adj", "normalize_adj_tensor", "propagate", "spmm",
    "KMeans", "MiniBatchKMeans", "ShardedKMeans", "shard_rows", "cluster_mean", "argmax_rows",
    "induced_subgraph", "group_by_label", "graph_sparse", "graph_compress", "ER_estimator", "attaw_ER_estimator",
]
