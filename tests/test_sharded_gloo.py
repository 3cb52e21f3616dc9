"""The multi-GPU path's distributed logic at world size 1 and 2 with the gloo backend on CPU
(SURVEY §8(e)): rows partitioned for the E-step / labels pass, clusters for the M-step / means.

The oracle's primitives stand in for the device ones (tests/sharded_util.OracleOps), so no GPU is
needed. Every result must be bit-identical across world sizes AND equal to scikit-learn's own
(fixture G3: KMeans with n_init 1 and 10 on the global RNG, the agents' call) — the partition only
changes who computes a value, never how.
"""
import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _paths():
    for p in (ROOT, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"), HERE):
        if p not in sys.path:
            sys.path.insert(0, p)


def _worker(rank, world, port, job, out_dir):
    _paths()
    import torch
    import torch.distributed as dist
    from gdd import sharded
    from sharded_util import OracleOps, init_gloo
    from oracle import oracle as O
    init_gloo(rank, world, port)
    ops = OracleOps()
    kind, args = job
    res = {}
    if kind == "kmeans":
        X, k, n_init, seed = args[:4]
        split = args[4] if len(args) > 4 else False
        if seed is None:
            np.random.seed(15)
        m = sharded.ShardedKMeans(n_clusters=k, n_init=n_init, random_state=seed, ops=ops,
                                  split_columns=split).fit(X)
        res = dict(labels=m.labels_, centers=m.cluster_centers_, n_iter=m.n_iter_, inertia=m.inertia_)
    elif kind == "labels_mean":
        X, C, feat, k = args
        lab, sq, inertia = sharded.sharded_labels(torch.from_numpy(X), torch.from_numpy(C), ops=ops)
        fs, cnt = sharded.sharded_cluster_mean(torch.from_numpy(feat), lab, k, ops=ops)
        fz, _ = sharded.sharded_cluster_mean(torch.from_numpy(feat), lab, k, empty_as_zero=True, ops=ops)
        res = dict(labels=lab.numpy(), sq=sq.numpy(), inertia=inertia, mean=fs.numpy(),
                   counts=cnt.numpy(), mean0=fz.numpy())
    elif kind == "minibatch":
        # MiniBatchKMeans as the multi-GPU path runs it: replicated steps (same RandomState on every
        # rank), then the partitioned final labels pass
        X, k = args
        r = O.minibatch_kmeans(X, k, random_state=15, batch_size=500, compute_labels=False)
        lab, sq, inertia = sharded.sharded_labels(torch.from_numpy(X),
                                                  torch.from_numpy(r["cluster_centers_"]), ops=ops)
        res = dict(labels=lab.numpy(), inertia=inertia, centers=r["cluster_centers_"])
    elif kind == "propagate":
        rowptr, col, val, X, T, alpha = args
        from gdd.graph import CSRGraph
        g = CSRGraph(torch.from_numpy(rowptr), torch.from_numpy(col), torch.from_numpy(val),
                     rowptr.shape[0] - 1)
        t, p = sharded.sharded_propagate(g, torch.from_numpy(X), T, alpha, ops=ops)
        res = dict(target=t.numpy(), p_last=p.numpy())
    elif kind == "pair":
        # distill_recsys's two kmeans_cluster calls split over the ranks (config 4): users on rank 0,
        # items on rank 1, broadcast from the owners; the oracle's scaler + Lloyd stand in for the fit
        Eu, Ei, ku, ki = args
        calls = []

        def fit(E, n_clusters, seed, minibatch, batch_size, n_init, device):
            calls.append(E.shape[0])
            Xs, _, _ = O.standard_scaler(E)
            r = O.kmeans(Xs, n_clusters, random_state=seed, n_init=n_init)
            return r["labels_"].astype(np.int64), r["cluster_centers_"].astype(np.float32)
        from gdd.pipeline import kmeans_cluster_pair
        (ul, uc), (il, ic) = kmeans_cluster_pair(Eu, Ei, ku, ki, seed=42, device="cpu",
                                                 group=dist.group.WORLD, fit=fit)
        res = dict(ul=ul, uc=uc, il=il, ic=ic)
        np.save(os.path.join(out_dir, f"calls{rank}.npy"), np.asarray(calls, np.int64))
    elif kind == "roles":
        # the inductive agent's three role propagations over the ranks (config 3)
        graphs, feats, T, alpha, shard = args
        if shard is not None:
            os.environ["GDD_SHARD_PROP"] = shard
        ops.normalize = lambda g: _oracle_norm(O, g)
        ops.propagate = lambda gn, X, T_, a: _oracle_prop(O, gn, X, T_, a)
        adjs = dict(graphs)
        fts = {r: torch.from_numpy(f) for r, f in feats.items()}
        gn, tg = sharded.propagate_roles(adjs, fts, T, alpha, group=dist.group.WORLD, ops=ops)
        res = {"norm_val": gn.values().numpy(), **{"t_" + r: tg[r].numpy() for r in tg}}
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **res)
    dist.destroy_process_group()


def _oracle_norm(O, A):
    import torch
    from gdd.graph import CSRGraph
    ro, co, vo = O.normalize_csr(A.indptr, A.indices, None, -1)
    return CSRGraph(torch.from_numpy(ro), torch.from_numpy(co), torch.from_numpy(vo), ro.shape[0] - 1)


def _oracle_prop(O, gn, X, T, alpha):
    import torch
    t, p = O.propagate(gn.rowptr.numpy(), gn.col.numpy(), gn.values().numpy(), X.numpy(), T, alpha)
    return torch.from_numpy(t), torch.from_numpy(p)


def _run(world, job, tmp):
    from sharded_util import free_port
    os.makedirs(tmp, exist_ok=True)
    mp.spawn(_worker, args=(world, free_port(), job, str(tmp)), nprocs=world, join=True)
    parts = [dict(np.load(os.path.join(tmp, f"r{r}.npz"))) for r in range(world)]
    for p in parts[1:]:  # every rank ends with the same result
        for key in p:
            assert np.array_equal(np.atleast_1d(p[key]).view(np.uint8), np.atleast_1d(parts[0][key]).view(np.uint8)), key
    return parts[0]


def _same(a, b):
    assert a.keys() == b.keys()
    for key in a:
        assert np.array_equal(np.atleast_1d(a[key]).view(np.uint8), np.atleast_1d(b[key]).view(np.uint8)), key


@pytest.mark.parametrize("n_init", [1, 10])
def test_sharded_lloyd_equals_sklearn_fixture(tmp_path, n_init):
    _paths()
    from golden_util import load
    z = load("golden_kmeans.npz")
    X = z["km_X"]
    one = _run(1, ("kmeans", (X, 70, n_init, None)), tmp_path / "w1")
    two = _run(2, ("kmeans", (X, 70, n_init, None)), tmp_path / "w2")
    _same(one, two)
    tag = f"km{n_init}"
    assert int(two["n_iter"]) == int(z[f"{tag}_n_iter"])
    assert np.array_equal(two["labels"], z[f"{tag}_labels"])
    assert np.array_equal(two["centers"].view(np.uint32), z[f"{tag}_centers"].view(np.uint32))
    assert float(two["inertia"]) == float(z[f"{tag}_inertia"])


@pytest.mark.parametrize("n,dim,k,world,split", [(3001, 8, 12, 2, False), (3001, 8, 12, 3, True),
                                                 (50, 4, 50, 2, False), (50, 4, 50, 3, True),
                                                 (300, 3, 12, 2, True), (300, 3, 12, 4, True)])
def test_sharded_lloyd_equals_oracle_incl_relocation(tmp_path, n, dim, k, world, split):
    # (50, 4, 50): duplicated rows and k = n, so clusters empty out and are relocated / copied;
    # with split_columns, world 3 splits 8 columns 3 + 3 + 2 and world 4 leaves a rank with no
    # column of dim 3
    _paths()
    from gdd import synth
    from oracle import oracle as O
    X = synth.blobs(n, dim, max(1, k // 3), seed=n)
    X[1::7] = X[0]
    ref = O.kmeans(X, k, random_state=7)
    one = _run(1, ("kmeans", (X, k, 1, 7)), tmp_path / "w1")
    two = _run(world, ("kmeans", (X, k, 1, 7, split)), tmp_path / f"w{world}")
    _same(one, two)
    assert int(two["n_iter"]) == ref["n_iter_"]
    assert np.array_equal(two["labels"], ref["labels_"])
    assert np.array_equal(two["centers"].view(np.uint32), ref["cluster_centers_"].view(np.uint32))
    assert float(two["inertia"]) == ref["inertia_"]


def test_sharded_labels_pass_and_cluster_means(tmp_path):
    _paths()
    from gdd import synth
    from oracle import oracle as O
    X = synth.blobs(4001, 40, 60, seed=3)
    C = X[:61].copy()
    C[17] += 1e4  # a centre nobody picks: an empty cluster (NaN mean, zero with empty_as_zero)
    feat = synth.features(4001, 33, 3)
    one = _run(1, ("labels_mean", (X, C, feat, 61)), tmp_path / "w1")
    two = _run(2, ("labels_mean", (X, C, feat, 61)), tmp_path / "w2")
    _same(one, two)
    lab, inertia = O.labels_inertia(X, C)
    assert np.array_equal(two["labels"], lab)
    assert float(two["inertia"]) == inertia
    ref, cnt = O.cluster_mean(feat, lab, 61)
    assert cnt[17] == 0
    assert np.array_equal(two["counts"], cnt)
    assert np.array_equal(two["mean"].view(np.uint32), ref.view(np.uint32))
    ref0, _ = O.cluster_mean(feat, lab, 61, empty_as_zero=True)
    assert np.array_equal(two["mean0"].view(np.uint32), ref0.view(np.uint32))


def test_sharded_minibatch_labels_equal_sklearn_order(tmp_path):
    _paths()
    from gdd import synth
    from oracle import oracle as O
    X = synth.blobs(6000, 12, 40, seed=8)
    ref = O.minibatch_kmeans(X, 40, random_state=15, batch_size=500)
    one = _run(1, ("minibatch", (X, 40)), tmp_path / "w1")
    two = _run(2, ("minibatch", (X, 40)), tmp_path / "w2")
    _same(one, two)
    assert np.array_equal(two["labels"], ref["labels_"])
    assert float(two["inertia"]) == ref["inertia_"]
    assert np.array_equal(two["centers"].view(np.uint32), ref["cluster_centers_"].view(np.uint32))


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("T", [1, 2, 5])
def test_sharded_propagate_equals_oracle(tmp_path, world, T):
    """Row-partitioned propagation (gdd.sharded.sharded_propagate): rank r computes rows
    [r*m, (r+1)*m) of each hop from the all-gathered previous hop; target and the last hop are
    bit-identical to the one-rank loop and the oracle's, with hub rows longer than one 256-entry
    segment, a ragged last shard (n % world != 0) and a rank-spanning degree skew."""
    _paths()
    import scipy.sparse as sp
    from gdd import synth
    from oracle import oracle as O
    n, d, alpha = 1201, 24, 0.91
    A = sp.csr_matrix(synth.chung_lu(n, 30.0, 11))
    A = A.tolil()
    A[3, :700] = 1  # a hub row spanning three segments
    A[:700, 3] = 1
    A = sp.csr_matrix(A)
    A.setdiag(0)
    A.eliminate_zeros()
    A.sort_indices()
    ro, co, vo = O.normalize_csr(A.indptr, A.indices, None, -1)
    assert np.diff(ro).max() > 512
    X = synth.features(n, d, 11)
    t_ref, p_ref = O.propagate(ro, co, vo, X, T, alpha)
    one = _run(1, ("propagate", (ro, co, vo, X, T, alpha)), tmp_path / "w1")
    many = _run(world, ("propagate", (ro, co, vo, X, T, alpha)), tmp_path / f"w{world}")
    _same(one, many)
    assert np.array_equal(many["target"].view(np.uint32), t_ref.view(np.uint32))
    assert np.array_equal(many["p_last"].view(np.uint32), p_ref.view(np.uint32))


def test_propagation_size_model():
    _paths()
    from gdd.sharded import propagation_shards_pay
    assert propagation_shards_pay(2449029, 130_000_000, 100, 8)    # ogbn-products: shard
    assert propagation_shards_pay(2449029, 130_000_000, 100, 2)
    assert not propagation_shards_pay(169343, 2_560_000, 128, 8)   # ogbn-arxiv: replicate
    assert not propagation_shards_pay(169343, 2_560_000, 128, 1)


def test_lloyd_size_model(monkeypatch):
    """lloyd_rows_pay (r06): the E-step's row-proportional part against the labels all-gather — the
    products Lloyd splits from two ranks (a ~0.23 ms bounded E-step per iteration), the recsys and
    Cora shapes replicate, one rank never splits, GDD_SHARD_LLOYD forces either."""
    _paths()
    from gdd.sharded import lloyd_rows_pay
    monkeypatch.delenv("GDD_SHARD_LLOYD", raising=False)
    assert all(lloyd_rows_pay(2449029, 47, 196, w) for w in (2, 4, 8))
    assert not lloyd_rows_pay(2449029, 47, 196, 1)
    assert not any(lloyd_rows_pay(n, 64, k, 8) for n, k in ((6040, 604), (3706, 371)))
    assert not lloyd_rows_pay(2708, 7, 70, 8)
    monkeypatch.setenv("GDD_SHARD_LLOYD", "0")
    assert not lloyd_rows_pay(2449029, 47, 196, 8)
    monkeypatch.setenv("GDD_SHARD_LLOYD", "1")
    assert lloyd_rows_pay(2708, 7, 70, 2) and not lloyd_rows_pay(2708, 7, 70, 1)


@pytest.mark.parametrize("world", [2, 3])
def test_recsys_pair_split_matches_one_rank(tmp_path, world):
    """kmeans_cluster_pair over a group (north star config 4): the users' fit runs on rank 0 only and
    the items' on rank 1 only (pair_owners), the results broadcast; every rank ends with the one-rank
    results bit for bit (oracle stand-in fits: StandardScaler + Lloyd, random_state 42)."""
    _paths()
    from gdd import synth
    Eu, Ei = synth.svd_like(700, 16, seed=1), synth.svd_like(450, 16, seed=2)
    one = _run(1, ("pair", (Eu, Ei, 70, 45)), tmp_path / "w1")
    many = _run(world, ("pair", (Eu, Ei, 70, 45)), tmp_path / f"w{world}")
    _same(one, many)
    calls = [np.load(tmp_path / f"w{world}" / f"calls{r}.npy").tolist() for r in range(world)]
    assert calls[0] == [700] and calls[1] == [450] and all(c == [] for c in calls[2:])
    assert np.load(tmp_path / "w1" / "calls0.npy").tolist() == [700, 450]


def _role_graphs(n=900, seed=4):
    """A GraphSAINT-style split: the induced train/val/test sub-graphs of one Chung-Lu graph."""
    import scipy.sparse as sp
    from gdd import synth
    A = sp.csr_matrix(synth.chung_lu(n, 20.0, seed))
    rs = np.random.RandomState(seed)
    perm = rs.permutation(n)
    idx = {"train": np.sort(perm[:600]), "val": np.sort(perm[600:700]), "test": np.sort(perm[700:])}
    X = synth.features(n, 12, seed)
    graphs = {r: sp.csr_matrix(A[np.ix_(i, i)]) for r, i in idx.items()}
    for g in graphs.values():
        g.sort_indices()
    feats = {r: np.ascontiguousarray(X[i]) for r, i in idx.items()}
    return graphs, feats


@pytest.mark.parametrize("world,shard", [(2, None), (3, None), (4, "1"), (4, "0")])
def test_role_propagations_split_matches_one_rank(tmp_path, world, shard):
    """propagate_roles (north star config 3): train on rank 0 (row-partitioned over ranks 0 and 3 at
    world 4 when forced), val on rank 1, test on rank 2 (rank 1 at world 2), targets broadcast —
    every rank holds the one-rank targets and normalised train graph bit for bit, equal to the
    oracle's loops."""
    _paths()
    from oracle import oracle as O
    graphs, feats = _role_graphs()
    T, alpha = 5, 0.9
    one = _run(1, ("roles", (graphs, feats, T, alpha, None)), tmp_path / "w1")
    many = _run(world, ("roles", (graphs, feats, T, alpha, shard)), tmp_path / f"w{world}")
    _same(one, many)
    for r, g in graphs.items():
        ro, co, vo = O.normalize_csr(g.indptr, g.indices, None, -1)
        t_ref, _ = O.propagate(ro, co, vo, feats[r], T, alpha)
        assert np.array_equal(many["t_" + r].view(np.uint32), t_ref.view(np.uint32)), r


def test_role_and_pair_owners():
    _paths()
    from gdd.sharded import pair_owners, role_owners
    assert pair_owners(1) == (0, 0) and pair_owners(2) == (0, 1) and pair_owners(8) == (0, 1)
    assert role_owners(1) == {"train": [0], "val": [0], "test": [0]}
    assert role_owners(2) == {"train": [0], "val": [1], "test": [1]}
    assert role_owners(3) == {"train": [0], "val": [1], "test": [2]}
    assert role_owners(8) == {"train": [0, 3, 4, 5, 6, 7], "val": [1], "test": [2]}
