"""The reference's hot-path call sites as single functions (drop-ins for the agents and the recsys CLI).

* :func:`pretrained_clustering_hot_path` — the path of ``ClustGDD.pretrained_clustering``
  (clustgdd_agent_transduct.py:38-129): normalise the adjacency, propagate, cluster the caller's
  logits (MiniBatchKMeans for ogbn-arxiv, KMeans otherwise), per-cluster feature means and argmax
  labels. The MLP that produces the logits (models/gcn.py:626-653) is the caller's: pass the
  logits, or a callable that maps ``target_feat`` to them.
* :func:`pretrained_clustering_induct_hot_path` — the inductive agent's path
  (clustgdd_agent_induct.py:37-155): the same stages per role sub-graph (train/val/test), k-means on
  the train logits (MiniBatchKMeans for reddit, KMeans otherwise); :func:`graphsaint_split` builds
  its inputs as ``utils_graphsaint.DataGraphSAINT`` does (induced sub-graphs, train-fitted scaler).
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
from .graph import CSRGraph, induced_subgraph, normalize_adj, propagate, to_csr
from .kmeans import KMeans, MiniBatchKMeans


def _lloyd(n_clusters, group, **kw):
    """KMeans on one GPU, or gdd.sharded.ShardedKMeans (rows/clusters partitioned, bit-identical)
    when `group` spans several ranks."""
    from .sharded import ShardedKMeans, world_of
    if group is not None and world_of(group)[1] > 1:
        return ShardedKMeans(n_clusters=n_clusters, group=group, **kw)
    return KMeans(n_clusters=n_clusters, **kw)


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


def standard_scaler_transform(X, mean: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    """StandardScaler.transform with a fitted (mean_, scale_) (fp64 device vectors)."""
    lib = _lib.device_lib()
    Xd = X.to(dtype=torch.float32).contiguous()
    out = torch.empty_like(Xd)
    _lib.check(lib.gdd_standard_scaler_transform(Xd.shape[0], Xd.shape[1], Xd.data_ptr(),
                                                 mean.data_ptr(), scale.data_ptr(), out.data_ptr(),
                                                 _lib.stream_ptr(Xd.device)))
    return out


def graphsaint_split(adj_full, feat, idx_train, idx_val, idx_test, device="cuda"):
    """The preparation of ``utils_graphsaint.DataGraphSAINT`` (utils_graphsaint.py:17-50) on the
    device, from the already-loaded ``adj_full`` and raw ``feats``: the three induced sub-graphs
    ``adj_full[np.ix_(idx, idx)]`` and the features standardised with a StandardScaler fitted on
    the train rows (then ``feat[idx]`` per role). Role lists must be strictly increasing (the
    GraphSAINT role.json lists are). Returns a namespace with the reference's attribute names
    (adj_full, feat_full, feat_train/val/test, adj_train/val/test, idx_train/val/test); graphs are
    :class:`CSRGraph`, features device fp32. (The ogbn-arxiv symmetrisation at :19-21 is a
    file-format fix-up of one dataset and is left to the loader.)
    """
    from types import SimpleNamespace
    g = adj_full if isinstance(adj_full, CSRGraph) else to_csr(adj_full, device=device)
    X = feat if isinstance(feat, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(feat, np.float32))
    X = X.to(device=g.device, dtype=torch.float32).contiguous()
    ids = {}
    for name, idx in (("train", idx_train), ("val", idx_val), ("test", idx_test)):
        t = idx if isinstance(idx, torch.Tensor) else torch.from_numpy(np.asarray(idx, np.int64))
        ids[name] = t.to(device=g.device, dtype=torch.int64)
    _, mean, scale = standard_scaler(X.index_select(0, ids["train"]), device=g.device)  # :40-42
    feat_full = standard_scaler_transform(X, mean, scale)                                # :43
    ns = SimpleNamespace(adj_full=g, feat_full=feat_full, scaler_mean=mean, scaler_scale=scale)
    for name, t in ids.items():
        setattr(ns, "idx_" + name, t)
        setattr(ns, "feat_" + name, feat_full.index_select(0, t))                         # :46-48
        setattr(ns, "adj_" + name, induced_subgraph(g, t))                                 # :34-36
    return ns


def load_graphsaint(dataset_dir: str, dataset: str = "", device="cuda"):
    """utils_graphsaint.DataGraphSAINT(dataset) (utils_graphsaint.py:14-68) from a GraphSAINT-format
    directory (adj_full.npz, role.json, feats.npy, class_map.json): the files are read on the host
    with loaders that execute nothing (scipy.sparse.load_npz / numpy.load without pickles / json),
    then :func:`graphsaint_split` prepares the role sub-graphs and the train-fitted scaling on the
    device. Labels follow process_labels (:70-87): a list per node gives a multi-label matrix, ints a
    vector shifted to start at 0. ogbn-arxiv is symmetrised as in :19-21."""
    import json
    import os
    import scipy.sparse as sp
    adj_full = sp.load_npz(os.path.join(dataset_dir, "adj_full.npz")).tocsr()
    if dataset == "ogbn-arxiv":
        adj_full = adj_full + adj_full.T
        adj_full[adj_full > 1] = 1
    with open(os.path.join(dataset_dir, "role.json")) as f:
        role = json.load(f)
    feat = np.load(os.path.join(dataset_dir, "feats.npy"), allow_pickle=False)
    with open(os.path.join(dataset_dir, "class_map.json")) as f:
        class_map = json.load(f)
    n = adj_full.shape[0]
    first = next(iter(class_map.values()))
    if isinstance(first, list):
        labels = np.zeros((n, len(first)))
        for k_, v in class_map.items():
            labels[int(k_)] = v
        nclass = len(first)
    else:
        labels = np.zeros(n, dtype=np.int32)
        for k_, v in class_map.items():
            labels[int(k_)] = v
        labels = labels - labels.min()
        nclass = int(labels.max()) + 1
    ns = graphsaint_split(adj_full, feat, role["tr"], role["va"], role["te"], device=device)
    ns.nnodes, ns.nclass, ns.labels_full = n, nclass, labels
    for name, key in (("train", "tr"), ("val", "va"), ("test", "te")):
        setattr(ns, "labels_" + name, labels[np.asarray(role[key], dtype=np.int64)])
    return ns


def kmeans_cluster(X, n_clusters: int, seed: int, minibatch: bool = True, batch_size: int = 2048,
                   device="cuda", n_init="auto", group=None):
    """distill_recsys.kmeans_cluster on the device -> (labels int64 numpy, centres fp32 numpy).
    The reference passes ``n_init="auto"`` explicitly (distill_recsys.py:176-178), the default here."""
    if n_clusters <= 0:
        raise ValueError("n_clusters must be > 0")
    n = X.shape[0]
    if n_clusters >= n:
        n_clusters = max(1, min(n_clusters, n))
    Xs, _, _ = standard_scaler(X, device=device)
    if minibatch and n > 20000:
        km = MiniBatchKMeans(n_clusters=n_clusters, random_state=seed, batch_size=batch_size,
                             n_init=n_init, device=device, group=group)
    else:
        km = _lloyd(n_clusters, group, random_state=seed, n_init=n_init, device=device)
    km.fit(Xs)
    return km.labels_.astype(np.int64), km.cluster_centers_.astype(np.float32)


def kmeans_cluster_pair(user_emb, item_emb, n_user_clusters: int, n_item_clusters: int, seed: int,
                        minibatch: bool = True, batch_size: int = 2048, device="cuda", n_init="auto",
                        group=None, fit=None, concurrent: bool = True):
    """Both kmeans_cluster calls of distill_recsys's main (distill_recsys.py:569-583): users, then
    items -> ((u_labels int64, u_centres fp32), (i_labels, i_centres)), numpy.

    ``group`` (north star config 4, a torch.distributed group over the GPUs of a node): the two fits
    share nothing — each has its own ``random_state=seed`` — so the users' fit runs on rank 0 and the
    items' on rank 1 (one rank runs both when R = 1), and each result is broadcast from its owner
    (RCCL over xGMI). Every rank ends with the single-GPU results, bit for bit. ``fit`` (tests): a
    stand-in with kmeans_cluster's signature.

    One GPU (``concurrent``, r06): the two fits run side by side on two HIP streams, the items' fit
    from a second host thread. Their launches are latency-bound chains that fill a fraction of the
    CUs (k-means++ rounds of T x T workgroups, Lloyd iterations of a 6,040-row problem), so the GPU
    overlaps them; the library's host state is lock-protected and its error string thread-local,
    and each fit is the single-stream computation itself (the same bits)."""
    kw = dict(seed=seed, minibatch=minibatch, batch_size=batch_size, n_init=n_init)
    from .sharded import split_pair, world_of
    if group is None or world_of(group)[1] == 1:
        dev = torch.device(device)
        if fit is not None or not concurrent or dev.type != "cuda":
            fit = fit or kmeans_cluster
            return (fit(user_emb, n_clusters=n_user_clusters, device=device, **kw),
                    fit(item_emb, n_clusters=n_item_clusters, device=device, **kw))
        return _pair_two_streams(user_emb, item_emb, n_user_clusters, n_item_clusters, dev, kw)
    fit = fit or kmeans_cluster
    jobs = []
    for E, k in ((user_emb, n_user_clusters), (item_emb, n_item_clusters)):
        n, d = int(E.shape[0]), int(E.shape[1])
        k_eff = max(1, min(k, n)) if k >= n else k  # kmeans_cluster's clamp
        if k <= 0:
            raise ValueError("n_clusters must be > 0")
        spec = [((n,), torch.int64), ((k_eff, d), torch.float32)]
        jobs.append((lambda E=E, k=k: fit(E, n_clusters=k, device=device, **kw), spec))
    (ul, uc), (il, ic) = split_pair(jobs, group=group, device=device)
    return ((ul.cpu().numpy(), uc.cpu().numpy()), (il.cpu().numpy(), ic.cpu().numpy()))


def _pair_two_streams(user_emb, item_emb, ku: int, ki: int, dev, kw):
    """kmeans_cluster(users) on one stream of this thread, kmeans_cluster(items) on another stream
    from a helper thread; both ordered after the caller's stream, and the caller's stream after both."""
    import threading
    cur = torch.cuda.current_stream(dev)
    streams = (torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev))
    out, err = [None, None], [None, None]

    def run(j, E, k):
        try:
            with torch.cuda.device(dev), torch.cuda.stream(streams[j]):
                streams[j].wait_stream(cur)
                out[j] = kmeans_cluster(E, n_clusters=k, device=dev, **kw)
        except BaseException as e:  # re-raised on the caller's thread
            err[j] = e

    helper = threading.Thread(target=run, args=(1, item_emb, ki))
    helper.start()
    run(0, user_emb, ku)
    helper.join()
    for s in streams:
        cur.wait_stream(s)
    for e in err:
        if e is not None:
            raise e
    return out[0], out[1]


def teacher_means(emb: torch.Tensor, assignment, num_clusters: int) -> torch.Tensor:
    """index_add_ / bincount.clamp_min(1) super-node means (empty cluster -> zero row)."""
    out, _ = cluster_mean(emb.to(torch.float32), assignment, num_clusters, empty_as_zero=True)
    return out


def pretrained_clustering_hot_path(features, adj, T: int, alpha: float, logits, nnodes_syn: int,
                                   dataset: str = "", seed: int = 15, cluster_minibatch: int = 1000,
                                   device="cuda", n_init="auto", group=None):
    """The hot path of ClustGDD.pretrained_clustering.

    ``group``: a torch.distributed group over the GPUs of one node — the graph is distilled once,
    with the k-means rows and the cluster means partitioned over the ranks (gdd.sharded), results
    bit-identical to one GPU.

    ``n_init``: the estimators' default. The reference constructs them without ``n_init``
    (transduct:103,105), so the count is the installed scikit-learn's default: 1 under >= 1.4
    ('auto', what the fixtures were made with), 10 (KMeans) / 3 (MiniBatchKMeans) under the 1.3.2
    that ``ClustGDD/README.md`` pins. Pass ``n_init=10`` (or 3) to reproduce 1.3.2.

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
    target_feat, prop_feat = propagate(adj_norm, X, T, alpha, group=group)  # transduct:59-65
    out = logits(target_feat) if callable(logits) else logits
    if dataset == "ogbn-arxiv":                                  # transduct:102-105
        km = MiniBatchKMeans(n_clusters=nnodes_syn, random_state=seed, n_init=n_init,
                             batch_size=cluster_minibatch, device=device, group=group).fit(out)
    else:
        km = _lloyd(nnodes_syn, group, n_init=n_init, device=device).fit(out)
    feat_syn, _ = cluster_mean(target_feat, km.labels_device_, nnodes_syn, group=group)  # :121-125
    labels_syn = argmax_rows(km.cluster_centers_device_)                    # transduct:126
    return feat_syn, labels_syn, km.labels_device_.to(torch.int32), adj_norm, target_feat, prop_feat


def pretrained_clustering_induct_hot_path(data, T: int, alpha: float, logits_train, nnodes_syn: int,
                                          dataset: str = "", seed: int = 15,
                                          cluster_minibatch: int = 1000, device="cuda",
                                          n_init="auto", group=None, phases=None):
    """The hot path of the inductive ClustGDD.pretrained_clustering (clustgdd_agent_induct.py:37-155).
    ``n_init`` as in :func:`pretrained_clustering_hot_path` (induct:131-134 passes none).

    ``data`` carries ``adj_train/adj_val/adj_test`` (CSRGraph or anything :func:`to_csr` takes) and
    ``feat_train/feat_val/feat_test`` (e.g. :func:`graphsaint_split`'s result). ``logits_train``: the
    MLP's train-node output (n_train x C), or a callable ``f(target_train, target_val) -> logits``
    (the MLP is fitted on both, :103-109). Each role graph is normalised and propagated on its own
    (:56-94); k-means runs on the train logits — MiniBatchKMeans(random_state=seed) for 'reddit',
    KMeans on the global numpy RNG otherwise (:129-134) — and the cluster means are taken over the
    train targets (:143-154). Returns (cluster_feat_centers, cluster_center_labels, cluster_labels
    int32, target_feat_train, adj_train_norm, target_feat_val, target_feat_test).

    ``group``: the three role propagations run on different ranks (train on rank 0 — row-partitioned
    over ranks 0, 3, 4, ... where that pays — val on rank 1, test on rank 2), their targets broadcast;
    the k-means labels pass and the cluster means are partitioned as in the transductive path.
    Bit-identical to one GPU. ``phases`` (optional dict): synchronised wall ms per stage on this rank.
    """
    from .sharded import DeviceOps, propagate_roles
    adjs, feats = {}, {}
    dev = torch.device(device)
    for name in ("train", "val", "test"):
        adjs[name] = getattr(data, "adj_" + name)
        X = getattr(data, "feat_" + name)
        X = X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(X, np.float32))
        if isinstance(adjs[name], CSRGraph):
            dev = adjs[name].device
        feats[name] = X.to(device=dev, dtype=torch.float32).contiguous()
    # :56-94 — each role graph normalised and propagated on its own; with a group the three loops
    # run on different ranks (gdd.sharded.role_owners) and the targets are broadcast
    norm_train, targets = propagate_roles(adjs, feats, T, alpha, group=group, ops=DeviceOps(dev),
                                          phases=phases)
    norms = {"train": norm_train}
    import time
    t_prev = [time.perf_counter()]

    def mark(name):
        if phases is not None:
            torch.cuda.synchronize(dev)
            now = time.perf_counter()
            phases[name] = (now - t_prev[0]) * 1e3
            t_prev[0] = now

    mark("broadcast_targets_wait")
    out = logits_train(targets["train"], targets["val"]) if callable(logits_train) else logits_train
    mark("logits")
    if dataset == "reddit":                                                         # :129-134
        km = MiniBatchKMeans(n_clusters=nnodes_syn, random_state=seed, batch_size=cluster_minibatch,
                             n_init=n_init, device=device, group=group).fit(out)
    else:
        km = _lloyd(nnodes_syn, group, n_init=n_init, device=device).fit(out)
    mark("kmeans")
    feat_syn, _ = cluster_mean(targets["train"], km.labels_device_, nnodes_syn, group=group)     # :143-151
    labels_syn = argmax_rows(km.cluster_centers_device_)                            # :152
    mark("cluster_mean")
    return (feat_syn, labels_syn, km.labels_device_.to(torch.int32), targets["train"], norms["train"],
            targets["val"], targets["test"])
