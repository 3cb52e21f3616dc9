"""gdd — MI355X-native hot path of ClustGDD graph distillation.

Drop-in replacements for the reference's hot-path call sites (see include/gdd.h for the C ABI and
the reference file:line each entry point replaces):

* :func:`gdd.graph.to_csr`, :func:`gdd.graph.normalize_adj_tensor`, :func:`gdd.graph.propagate`
* :class:`gdd.kmeans.KMeans`, :class:`gdd.kmeans.MiniBatchKMeans`
* :func:`gdd.cluster.cluster_mean`, :func:`gdd.cluster.argmax_rows`
* :func:`gdd.pipeline.pretrained_clustering_hot_path` — normalise → propagate → k-means on the
  logits → cluster means → argmax labels, as ClustGDD.pretrained_clustering does it.
"""
from . import _lib  # noqa: F401  (imports torch first, see _lib docstring)
from .cluster import argmax_rows, cluster_mean, group_by_label
from .graph import CSRGraph, normalize_adj, normalize_adj_tensor, propagate, spmm, to_csr
from .kmeans import KMeans, MiniBatchKMeans

__all__ = [
    "CSRGraph", "to_csr", "normalize_adj", "normalize_adj_tensor", "propagate", "spmm",
    "KMeans", "MiniBatchKMeans", "cluster_mean", "argmax_rows", "group_by_label",
]
