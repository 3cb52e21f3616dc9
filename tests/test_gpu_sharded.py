"""The multi-GPU path on the device primitives (gdd.sharded): one rank equals gdd.KMeans and the
sklearn fixtures bit for bit; two ranks (two processes sharing cuda:0 over gloo — RCCL needs one GPU
per rank, and this box has one) equal one rank for ShardedKMeans, the partitioned MiniBatchKMeans
labels pass and the partitioned cluster means."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import gdd  # noqa: E402
from gdd import synth  # noqa: E402
from gdd.sharded import ShardedKMeans  # noqa: E402
from golden_util import load  # noqa: E402
from sharded_util import free_port  # noqa: E402


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_one_rank_equals_kmeans_and_sklearn():
    z = load("golden_kmeans.npz")
    X = z["km_X"]
    np.random.seed(15)
    s = ShardedKMeans(n_clusters=70, n_init=10, device="cuda:0").fit(X)
    np.random.seed(15)
    m = gdd.KMeans(n_clusters=70, n_init=10).fit(X)
    assert s.n_iter_ == m.n_iter_ == int(z["km10_n_iter"])
    assert np.array_equal(s.labels_, m.labels_) and np.array_equal(s.labels_, z["km10_labels"])
    assert np.array_equal(_bits(s.cluster_centers_), _bits(z["km10_centers"]))
    assert s.inertia_ == m.inertia_ == float(z["km10_inertia"])


def _worker(rank, world, port, X, Xm, feat, out):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE),
                                                          "graph-distillation-for-recommendation_amd"), HERE]
    os.environ["GDD_SHARD_LLOYD"] = "1"  # the phase loop (the size model would replicate here)
    import torch.distributed as dist
    import gdd as G
    from gdd.sharded import ShardedKMeans as SK
    from sharded_util import init_gloo
    init_gloo(rank, world, port)
    g = dist.group.WORLD
    np.random.seed(15)
    m = SK(n_clusters=40, device="cuda:0", group=g, split_columns=True).fit(X)  # pipelines: False
    mb = G.MiniBatchKMeans(n_clusters=30, random_state=15, batch_size=500, device="cuda:0", group=g).fit(Xm)
    fs, cnt = G.cluster_mean(torch.from_numpy(feat).cuda(), mb.labels_device_, 30, group=g)
    np.savez(os.path.join(out, f"r{rank}.npz"), labels=m.labels_, centers=m.cluster_centers_,
             n_iter=m.n_iter_, inertia=m.inertia_, mb_labels=mb.labels_, mb_inertia=mb.inertia_,
             mb_centers=mb.cluster_centers_, mean=fs.cpu().numpy(), counts=cnt.cpu().numpy())
    dist.destroy_process_group()


def test_two_ranks_match_one():
    X = synth.blobs(20000, 24, 40, seed=4)
    X[1::9] = X[0]
    Xm = synth.blobs(12000, 16, 30, seed=6)
    feat = synth.features(12000, 100, 6)
    np.random.seed(15)
    one = gdd.KMeans(n_clusters=40).fit(X)
    mb = gdd.MiniBatchKMeans(n_clusters=30, random_state=15, batch_size=500).fit(Xm)
    fs, cnt = gdd.cluster_mean(torch.from_numpy(feat).cuda(), mb.labels_device_, 30)
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"gdd_sharded_{os.getpid()}")
    os.makedirs(out, exist_ok=True)
    mp.spawn(_worker, args=(2, free_port(), X, Xm, feat, out), nprocs=2, join=True)
    for r in range(2):
        p = np.load(os.path.join(out, f"r{r}.npz"))
        assert int(p["n_iter"]) == one.n_iter_
        assert np.array_equal(p["labels"], one.labels_)
        assert np.array_equal(_bits(p["centers"]), _bits(one.cluster_centers_))
        assert float(p["inertia"]) == one.inertia_
        assert np.array_equal(p["mb_labels"], mb.labels_)
        assert float(p["mb_inertia"]) == mb.inertia_
        assert np.array_equal(_bits(p["mb_centers"]), _bits(mb.cluster_centers_))
        assert np.array_equal(p["counts"], cnt.cpu().numpy())
        assert np.array_equal(_bits(p["mean"]), _bits(fs.cpu().numpy()))


def _pipelines(group, A, feat, logits, ind, logits_tr, E):
    """The three hot-path entry points (transductive / inductive pretrained clustering, the recsys
    kmeans_cluster), each with a MiniBatchKMeans and a Lloyd dataset branch."""
    from gdd.pipeline import (kmeans_cluster, pretrained_clustering_hot_path,
                              pretrained_clustering_induct_hot_path)
    out = {}
    for ds in ("ogbn-arxiv", "cora"):
        np.random.seed(15)
        fs, ls, cl = pretrained_clustering_hot_path(feat, A, 4, 0.8, logits, 60, dataset=ds, seed=15,
                                                    cluster_minibatch=500, device="cuda:0", group=group)[:3]
        out.update({f"{ds}_fs": fs.cpu().numpy(), f"{ds}_ls": ls.cpu().numpy(), f"{ds}_cl": cl.cpu().numpy()})
    for ds in ("reddit", "flickr"):
        np.random.seed(15)
        fs, ls, cl = pretrained_clustering_induct_hot_path(ind, 3, 0.8, logits_tr, 40, dataset=ds, seed=15,
                                                           cluster_minibatch=300, device="cuda:0",
                                                           group=group)[:3]
        out.update({f"{ds}_fs": fs.cpu().numpy(), f"{ds}_ls": ls.cpu().numpy(), f"{ds}_cl": cl.cpu().numpy()})
    lab, cen = kmeans_cluster(E, n_clusters=150, seed=42, minibatch=False, device="cuda:0", group=group)
    out.update(rs_labels=lab, rs_centers=cen)
    # config 4's pair split: users on rank 0, items on rank 1, broadcast (one rank: both in turn)
    from gdd.pipeline import kmeans_cluster_pair
    (ul, uc), (il, ic) = kmeans_cluster_pair(E, E[:1700] * 0.5 + 0.25, 150, 90, seed=42, minibatch=False,
                                             device="cuda:0", group=group)
    out.update(pair_ul=ul, pair_uc=uc, pair_il=il, pair_ic=ic)
    return out


def _pipeline_inputs():
    from gdd import data as D
    d = D.synthetic("cora", seed=5, d=48)
    A = d.adj_full
    logits = synth.linear_logits(d.feat_full, 7, 5)
    logits_tr = synth.linear_logits(d.feat_train + 0.5, 7, 6)
    E = synth.svd_like(3000, 32, seed=3)
    return A, d.feat_full, logits, d, logits_tr, E


def _pipeline_worker(rank, world, port, out):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE),
                                                          "graph-distillation-for-recommendation_amd"), HERE]
    os.environ["GDD_SHARD_LLOYD"] = "1"  # the phase loop (the size model would replicate here)
    import torch.distributed as dist
    import gdd as G
    from sharded_util import init_gloo
    init_gloo(rank, world, port)
    res = _pipelines(dist.group.WORLD, *_pipeline_inputs())
    # with a process group up but group=None, each rank fits its own data on its own
    own = G.MiniBatchKMeans(n_clusters=25, random_state=15, batch_size=400).fit(
        synth.blobs(5000 + 1000 * rank, 12, 25, seed=100 + rank))
    res.update(own_labels=own.labels_, own_inertia=own.inertia_)
    np.savez(os.path.join(out, f"p{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_two_ranks_pipelines_match_one(world):
    """pretrained_clustering_hot_path, pretrained_clustering_induct_hot_path, kmeans_cluster and
    kmeans_cluster_pair with a two- and a three-rank group (MiniBatchKMeans: partitioned labels pass;
    Lloyd: ShardedKMeans; cluster means by cluster slices; the inductive role graphs propagated on
    different ranks and broadcast; the recsys pair's fits on ranks 0 and 1) give one rank's outputs bit
    for bit; and MiniBatchKMeans(group=None) inside an initialised process group stays a single-rank
    fit on each rank's own data."""
    one = _pipelines(None, *_pipeline_inputs())
    own = [gdd.MiniBatchKMeans(n_clusters=25, random_state=15, batch_size=400).fit(
        synth.blobs(5000 + 1000 * r, 12, 25, seed=100 + r)) for r in range(world)]
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"gdd_pipes_{os.getpid()}_{world}")
    os.makedirs(out, exist_ok=True)
    mp.spawn(_pipeline_worker, args=(world, free_port(), out), nprocs=world, join=True)
    for r in range(world):
        p = np.load(os.path.join(out, f"p{r}.npz"))
        for key, v in one.items():
            a, b = np.ascontiguousarray(p[key]), np.ascontiguousarray(v)
            assert a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8)), key
        assert np.array_equal(p["own_labels"], own[r].labels_) and float(p["own_inertia"]) == own[r].inertia_


def _prop_worker(rank, world, port, rowptr, col, X, T, alpha, out):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE),
                                                          "graph-distillation-for-recommendation_amd"), HERE]
    os.environ["GDD_SHARD_PROP"] = "1"  # the size model would replicate at this test's size
    import scipy.sparse as sp
    import torch.distributed as dist
    import gdd as G
    from sharded_util import init_gloo
    init_gloo(rank, world, port)
    A = sp.csr_matrix((np.ones(col.shape[0], np.float32), col, rowptr), shape=(X.shape[0],) * 2)
    gn = G.normalize_adj(G.to_csr(A, device="cuda:0"))
    t, p = G.propagate(gn, torch.from_numpy(X).cuda(), T, alpha, group=dist.group.WORLD)
    np.savez(os.path.join(out, f"g{rank}.npz"), target=t.cpu().numpy(), p_last=p.cpu().numpy())
    dist.destroy_process_group()


def _lloyd_rows_worker(rank, world, port, X, out):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE),
                                                          "graph-distillation-for-recommendation_amd"), HERE]
    os.environ["GDD_SHARD_LLOYD"] = "1"
    import torch.distributed as dist
    from gdd.sharded import ShardedKMeans as SK
    from sharded_util import init_gloo
    init_gloo(rank, world, port)
    m = SK(n_clusters=60, random_state=15, device="cuda:0", group=dist.group.WORLD).fit(X)
    np.savez(os.path.join(out, f"l{rank}.npz"), labels=m.labels_, centers=m.cluster_centers_,
             n_iter=m.n_iter_, inertia=m.inertia_, mode=m.mode_)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_lloyd_rows_products_path_matches_one(world):
    """ShardedKMeans' row split on the products-shape code path (r06: the size model now splits config
    5's Lloyd at N > 1): >= 65,536 rows at dim 47, so the fold and the bounded E-step's row lists read
    the zero-padded copy of X; bit-identical to gdd.KMeans on one rank."""
    n, dim = 100003, 47
    rng = np.random.default_rng(8)
    X = (rng.standard_normal((n, 32)) @ rng.standard_normal((32, dim)) / 5.0 + rng.standard_normal(dim)).astype(np.float32)
    one = gdd.KMeans(n_clusters=60, random_state=15).fit(X)
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"gdd_lrows_{os.getpid()}_{world}")
    os.makedirs(out, exist_ok=True)
    mp.spawn(_lloyd_rows_worker, args=(world, free_port(), X, out), nprocs=world, join=True)
    for r in range(world):
        p = np.load(os.path.join(out, f"l{r}.npz"))
        assert str(p["mode"]) == "rows"
        assert int(p["n_iter"]) == one.n_iter_
        assert np.array_equal(p["labels"], one.labels_)
        assert np.array_equal(_bits(p["centers"]), _bits(one.cluster_centers_))
        assert float(p["inertia"]) == one.inertia_


@pytest.mark.parametrize("world,T", [(2, 5), (3, 4)])
def test_ranks_row_partitioned_propagate_matches_one(world, T):
    """gdd.sharded.sharded_propagate on the device: rows partitioned over the ranks,
    one all-gather of each hop; target and the last hop bit-identical to gdd.propagate on one rank
    (d = 100 as ogbn-products, hub rows split over many segments, a ragged last shard)."""
    n, d, alpha = 30001, 100, 0.91
    A = synth.chung_lu(n, 40.0, 21).tocsr()
    A.sort_indices()
    assert np.diff(A.indptr).max() > 1024
    X = synth.features(n, d, 21)
    gn = gdd.normalize_adj(gdd.to_csr(A, device="cuda:0"))
    t1, p1 = gdd.propagate(gn, torch.from_numpy(X).cuda(), T, alpha)
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"gdd_prop_{os.getpid()}_{world}")
    os.makedirs(out, exist_ok=True)
    mp.spawn(_prop_worker, args=(world, free_port(), A.indptr.astype(np.int32), A.indices.astype(np.int32),
                                 X, T, alpha, out), nprocs=world, join=True)
    for r in range(world):
        p = np.load(os.path.join(out, f"g{r}.npz"))
        assert np.array_equal(_bits(p["target"]), _bits(t1.cpu().numpy()))
        assert np.array_equal(_bits(p["p_last"]), _bits(p1.cpu().numpy()))


def _nccl_worker(rank, world, port, X, feat, out):
    sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE),
                                                          "graph-distillation-for-recommendation_amd"), HERE]
    os.environ["GDD_SHARD_LLOYD"] = "1"
    os.environ["GDD_SHARD_PROP"] = "1"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    import gdd as G
    from gdd.sharded import ShardedKMeans as SK
    dev = torch.device("cuda", rank)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    g = dist.group.WORLD
    res = {}
    for split in (False, True):
        np.random.seed(15)
        m = SK(n_clusters=40, device=dev, group=g, split_columns=split).fit(X)
        res.update({f"labels{int(split)}": m.labels_, f"centers{int(split)}": m.cluster_centers_,
                    f"n_iter{int(split)}": m.n_iter_, f"inertia{int(split)}": m.inertia_})
    A = synth.chung_lu(6000, 12.0, 3)
    gn = G.normalize_adj(G.to_csr(A, device=dev))
    t, p = G.propagate(gn, torch.from_numpy(feat).to(dev), 5, 0.9, group=g)
    res.update(target=t.cpu().numpy(), p_last=p.cpu().numpy())
    np.savez(os.path.join(out, f"n{rank}.npz"), **res)
    dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="RCCL needs one GPU per rank (2 GPUs)")
def test_two_ranks_rccl_match_one():
    """the RCCL branches (in-place slot all-gathers of ShardedKMeans' phase loop, with and
    without the column split, and the row-partitioned propagation's per-hop all-gathers into the
    persistent buffers), two ranks on two GPUs, bit-identical to one GPU. Skipped on one-GPU boxes."""
    X = synth.blobs(20000, 24, 40, seed=4)
    X[1::9] = X[0]
    feat = synth.features(6000, 100, 6)
    np.random.seed(15)
    one = gdd.KMeans(n_clusters=40).fit(X)
    gn = gdd.normalize_adj(gdd.to_csr(synth.chung_lu(6000, 12.0, 3)))
    t1, p1 = gdd.propagate(gn, torch.from_numpy(feat).cuda(), 5, 0.9)
    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"gdd_rccl_{os.getpid()}")
    os.makedirs(out, exist_ok=True)
    mp.spawn(_nccl_worker, args=(2, free_port(), X, feat, out), nprocs=2, join=True)
    for r in range(2):
        p = np.load(os.path.join(out, f"n{r}.npz"))
        for s in ("0", "1"):
            assert int(p["n_iter" + s]) == one.n_iter_
            assert np.array_equal(p["labels" + s], one.labels_)
            assert np.array_equal(_bits(p["centers" + s]), _bits(one.cluster_centers_))
            assert float(p["inertia" + s]) == one.inertia_
        assert np.array_equal(_bits(p["target"]), _bits(t1.cpu().numpy()))
        assert np.array_equal(_bits(p["p_last"]), _bits(p1.cpu().numpy()))
