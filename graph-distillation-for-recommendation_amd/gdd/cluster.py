"""Per-cluster reductions of the ClustGDD hot path on MI355X.

* :func:`cluster_mean` replaces the k-launch Python loop of clustgdd_agent_transduct.py:116-125
  (``ft_source[torch.where(cluster_labels==i)[0]].mean(dim=0)`` for every i < k; induct :143-152)
  and the teacher ``index_add_``/``bincount`` means of distill_recsys.py:623-636
  (``empty_as_zero=True``: ``clamp_min(1)`` gives zero rows for empty clusters).
* :func:`argmax_rows` is ``torch.argmax(cluster_centers, dim=-1)`` (transduct:126).
A stable device counting sort groups the samples by label (no host round trip); every cluster row
is then one fp64 sum over its members in sample order, divided by the count and rounded to fp32
once. A label outside [0, k) belongs to no cluster, exactly as in the reference's ``labels == i``
loop over i < k.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def group_by_label(labels: torch.Tensor, k: int):
    """Stable grouping: (perm, offsets) with the samples of cluster c at perm[offsets[c]:offsets[c+1]]."""
    lib = _lib.device_lib()
    labels = labels.to(torch.int32).contiguous()
    n = labels.shape[0]
    dev = labels.device
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    offsets = torch.empty(k + 1, dtype=torch.int32, device=dev)
    ws = _lib.workspace(lib.gdd_group_ws_bytes(n, k), dev)
    _lib.check(lib.gdd_group_by_label(n, labels.data_ptr(), k, perm.data_ptr(), offsets.data_ptr(),
                                      ws.data_ptr(), ws.numel(), _lib.stream_ptr(dev)))
    return perm, offsets


def cluster_mean(feat: torch.Tensor, labels, k: int, empty_as_zero: bool = False, group=None):
    """Mean feature row of every cluster -> (feat_syn [k, d] fp32, counts [k] int64).

    An empty cluster gives a NaN row (the reference's mean over an empty selection) unless
    ``empty_as_zero``. ``group`` (a torch.distributed group with more than one rank): the clusters
    are partitioned over the ranks and the rows all-gathered (gdd.sharded; bit-identical).
    """
    lib = _lib.device_lib()
    feat = feat.contiguous()
    if feat.dtype != torch.float32:
        raise TypeError("feat must be float32")
    dev = feat.device
    if not isinstance(labels, torch.Tensor):
        labels = torch.from_numpy(np.asarray(labels))
    labels = labels.to(device=dev, dtype=torch.int32)
    n, d = feat.shape
    if labels.shape[0] != n:
        raise ValueError("labels and feat disagree on the number of samples")
    if group is not None:
        from .sharded import sharded_cluster_mean, world_of
        if world_of(group)[1] > 1:
            return sharded_cluster_mean(feat, labels, k, empty_as_zero=empty_as_zero, group=group)
    perm, offsets = group_by_label(labels, k)
    out = torch.empty((k, d), dtype=torch.float32, device=dev)
    counts = torch.empty(k, dtype=torch.int64, device=dev)
    _lib.check(lib.gdd_cluster_mean(n, d, feat.data_ptr(), perm.data_ptr(), offsets.data_ptr(), k,
                                    int(bool(empty_as_zero)), out.data_ptr(), counts.data_ptr(),
                                    _lib.stream_ptr(dev)))
    return out, counts


def argmax_rows(centers: torch.Tensor) -> torch.Tensor:
    lib = _lib.device_lib()
    centers = centers.to(torch.float32).contiguous()
    k, dim = centers.shape
    out = torch.empty(k, dtype=torch.int64, device=centers.device)
    _lib.check(lib.gdd_argmax_rows(k, dim, centers.data_ptr(), out.data_ptr(),
                                   _lib.stream_ptr(centers.device)))
    return out
