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
* :class:`gdd.sharded.ShardedKMeans` — Lloyd over range-partitioned rows on several ranks, one
  fixed-point all-reduce per iteration (rank-count invariant)
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
