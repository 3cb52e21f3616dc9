#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by running the REFERENCE code.

Runs only where /root/reference exists (the build container). It imports the reference's own
modules (ClustGDD/deep_robust_utils.py, clustgdd_agent_transduct.py, distill_recsys.py) with
in-memory stubs for the absent, off-path packages (torch_geometric, torch_sparse, ogb), executes
the hot-path code on small synthetic inputs, and saves inputs + outputs as .npz. No reference
source is copied; the fixtures are data. scikit-learn runs with one OpenMP/BLAS thread, the only
setting in which its Lloyd M-step merge order is deterministic.

  G1 golden_normalize.npz  deep_robust_utils.normalize_adj_tensor(sparse=True) on 4 graphs
  G2 golden_propagate.npz  the propagation loop (clustgdd_agent_transduct.py:59-65) in torch CPU
  G3 golden_kmeans.npz     MiniBatchKMeans / KMeans (n_init 1 and 10) / distill_recsys.kmeans_cluster
  G3b golden_kmeans_arxiv.json  MiniBatchKMeans on a 169,343 x 40 input (hashes of the outputs)
  G4/G5 golden_clustgdd_*.npz  ClustGDD.pretrained_clustering end to end (CPU), with the exact
                           k-means input and numpy RNG state captured at the sklearn call
  G6 golden_condense.npz   ClustGDD.graph_sparse(sp_type='attaw'/'vanilla'/'single') and
                           ClustGDD.graph_compress (clustgdd_agent_transduct.py:131-250), with the
                           effective-resistance intermediates of utils_clustgdd.attaw_ER_estimator
  G7 golden_clustgdd_induct_*.npz  the inductive pipeline: utils_graphsaint.DataGraphSAINT on files
                           written to a temp dir (StandardScaler on the train rows, the three
                           adj_full[np.ix_(idx, idx)] sub-graphs), then clustgdd_agent_induct
                           .ClustGDD.pretrained_clustering ('flickr': KMeans, 'reddit':
                           MiniBatchKMeans), with the k-means input and RNG state captured
  G9 golden_configs.npz / .json  config-shape k-means: KMeans(k=196)
                           on a 200,000 x 47 products-shaped input (global RNG after np.random.seed(15),
                           the agent's call) and distill_recsys.kmeans_cluster on ML-1M-shaped SVD
                           embeddings (6,040 users, k=604; 3,706 items, k=371; seed 42)
  G9b golden_full_shapes.json  MiniBatchKMeans(k=769, b=1000) on 153,932 x 41 and KMeans(k=196) on
                           the full 2,449,029 x 47 (config 3 / config 5 shapes), as hashes
  G10 golden_agent.npz  the reference ClustGDD transductive agent end to end on the CPU (train():
                           pretrained_clustering, graph_sparse('attaw'), graph_compress,
                           graph_refusion, then 5 x test_with_val) on gdd.data.synthetic('cora',
                           seed=15, d=300) with main_transduct.sh's Cora r=0.5 settings (postep cut
                           to 200): the k-means input, the pre-refusion cluster outputs, the
                           distilled graph, the torch RNG state before the GCN runs and the five
                           [train, test] accuracies. The agents call .cuda() in test_with_val; the
                           generator maps Tensor.cuda to the CPU for this run (no arithmetic change)
  G6r golden_alidisplay.npz  distill_recsys.main() on the real Rankformer/data/Ali-Display files
                           (a 20-epoch refine with artefacts, and the default 500-epoch run's stdout)
  G12 golden_agent_induct_{flickr,reddit}.npz  the reference inductive agent end to end on the CPU
                           (clustgdd_agent_induct.ClustGDD.train on DataGraphSAINT files: KMeans /
                           MiniBatchKMeans, graph_sparse('attaw'), graph_compress, the reweighted
                           graph_refusion, 5 x test_with_val), with the refusion inputs and both
                           torch RNG states captured, and stdout
  G8 golden_recsys.npz     distill_recsys.build_condensed_bipartite on synthetic interactions (with
                           empty super-nodes), condensed_csr_to_edge_index, and LightGCNCondensed
                           (propagate outputs, bpr_loss and every parameter gradient) on CPU
Usage: python tools/make_golden.py [G1 G2 ...]   (default: all)
"""
import hashlib
import json
import os
import sys
import types

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/ClustGDD"
OUT = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
from gdd import synth  # noqa: E402  (input generators only)


class _Stub(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return type(name, (), {})


def import_reference():
    for name in ["torch_geometric", "torch_geometric.nn", "torch_geometric.datasets",
                 "torch_geometric.transforms", "torch_geometric.utils", "torch_geometric.data",
                 "torch_geometric.loader", "torch_geometric.nn.conv", "torch_geometric.nn.inits",
                 "torch_geometric.typing", "torch_sparse", "torch_scatter", "ogb",
                 "ogb.nodeproppred", "deeprobust", "deeprobust.graph", "deeprobust.graph.utils"]:
        sys.modules.setdefault(name, _Stub(name))
    sys.path.insert(0, REF)
    import clustgdd_agent_transduct as agent
    import deep_robust_utils as du
    import distill_recsys as recsys
    return du, agent, recsys


def coo_sorted(t):
    t = t.coalesce()
    i = t.indices().numpy()
    v = t.values().numpy()
    o = np.lexsort((i[1], i[0]))
    return i[0][o].astype(np.int32), i[1][o].astype(np.int32), v[o].astype(np.float32)


def csr_arrays(A):
    A = sp.csr_matrix(A)
    A.sort_indices()
    return A.indptr.astype(np.int32), A.indices.astype(np.int32), A.data.astype(np.float32)


def g1_normalize(du):
    import torch  # noqa: F401
    out = {}
    base = synth.chung_lu(300, 6.0, 21)
    graphs = {"binary": base}
    g = base.tolil()
    g[0, 0] = 1.0
    g[3, 3] = 1.0
    graphs["selfloop0"] = sp.csr_matrix(g)  # A[0,0] != 0: fp32 path, no I added
    w = sp.csr_matrix(base).astype(np.float32)
    w.data = np.random.default_rng(5).uniform(0.25, 4.0, w.nnz).astype(np.float32)
    graphs["weighted"] = w
    iso = base.tolil()
    iso[7, :] = 0
    iso[:, 7] = 0
    graphs["isolated"] = sp.csr_matrix(iso)
    for name, A in graphs.items():
        A = sp.csr_matrix(A)
        A.eliminate_zeros()
        A.sort_indices()
        adj = du.sparse_mx_to_torch_sparse_tensor(A)
        r, c, v = coo_sorted(du.normalize_adj_tensor(adj, sparse=True))
        rp, ci, vi = csr_arrays(A)
        out.update({f"{name}_rowptr": rp, f"{name}_col": ci, f"{name}_val": vi,
                    f"{name}_out_row": r, f"{name}_out_col": c, f"{name}_out_val": v})
    np.savez_compressed(os.path.join(OUT, "golden_normalize.npz"), **out)


def g2_propagate(du):
    import torch
    out = {}
    A = synth.chung_lu(1000, 10.0, 22)
    X = synth.features(1000, 32, 22)
    rp, ci, vi = csr_arrays(A)
    out.update({"rowptr": rp, "col": ci, "val": vi, "X": X})
    adj_norm = du.normalize_adj_tensor(du.sparse_mx_to_torch_sparse_tensor(sp.csr_matrix(A)),
                                       sparse=True)
    for T, alpha in [(5, 0.8), (18, 0.91)]:
        features = torch.from_numpy(X)
        # the loop of clustgdd_agent_transduct.py:59-65, executed by torch on the CPU
        for t in range(T):
            if t == 0:
                prop_feat = features
                target_feat = (1 - alpha) * prop_feat
            else:
                prop_feat = alpha * adj_norm @ prop_feat
                target_feat = target_feat + (1 - alpha) * prop_feat
        out[f"target_T{T}"] = target_feat.numpy()
        out[f"prop_T{T}"] = prop_feat.numpy()
    np.savez_compressed(os.path.join(OUT, "golden_propagate.npz"), **out)


def g3_kmeans(recsys):
    from sklearn.cluster import KMeans, MiniBatchKMeans
    out = {}
    X = synth.blobs(5000, 40, 50, seed=31)
    m = MiniBatchKMeans(n_clusters=50, random_state=15, batch_size=1000).fit(X)
    out.update({"mb_X": X, "mb_labels": m.labels_.astype(np.int32),
                "mb_centers": m.cluster_centers_.astype(np.float32),
                "mb_n_steps": np.int64(m.n_steps_), "mb_inertia": np.float64(m.inertia_)})
    Xc = synth.blobs(2708, 7, 35, seed=32)
    for n_init in ("auto", 10):
        np.random.seed(15)  # KMeans(random_state=None) draws from the global RNG
        km = KMeans(n_clusters=70, n_init=n_init).fit(Xc)
        tag = "km1" if n_init == "auto" else "km10"
        out.update({f"{tag}_labels": km.labels_.astype(np.int32),
                    f"{tag}_centers": km.cluster_centers_.astype(np.float32),
                    f"{tag}_n_iter": np.int64(km.n_iter_), f"{tag}_inertia": np.float64(km.inertia_)})
    out["km_X"] = Xc
    # distill_recsys.kmeans_cluster (StandardScaler -> KMeans(random_state=42, n_init="auto"))
    E = synth.blobs(2000, 64, 100, seed=33)
    lab, cen = recsys.kmeans_cluster(E, n_clusters=200, seed=42, minibatch=False)
    out.update({"rs_X": E, "rs_labels": lab.astype(np.int64), "rs_centers": cen.astype(np.float32)})
    np.savez_compressed(os.path.join(OUT, "golden_kmeans.npz"), **out)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def g3b_arxiv():
    from sklearn.cluster import MiniBatchKMeans
    X = synth.blobs(169343, 40, 454, seed=34)
    m = MiniBatchKMeans(n_clusters=454, random_state=15, batch_size=1000).fit(X)
    rec = {"input": "gdd.synth.blobs(169343, 40, 454, seed=34)",
           "estimator": "MiniBatchKMeans(n_clusters=454, random_state=15, batch_size=1000)",
           "n_steps": int(m.n_steps_), "inertia": float(m.inertia_),
           "labels_sha256": sha(m.labels_.astype(np.int32)),
           "centers_sha256": sha(m.cluster_centers_.astype(np.float32))}
    with open(os.path.join(OUT, "golden_kmeans_arxiv.json"), "w") as f:
        json.dump(rec, f, indent=1)


def g9_configs(recsys):
    from sklearn.cluster import KMeans
    X = synth.blobs(200000, 47, 196, seed=5)
    np.random.seed(15)
    m = KMeans(n_clusters=196).fit(X)
    rec = {"products_input": "gdd.synth.blobs(200000, 47, 196, seed=5)",
           "products_estimator": "np.random.seed(15); KMeans(n_clusters=196) (random_state=None)",
           "products_n_iter": int(m.n_iter_), "products_inertia": float(m.inertia_),
           "products_labels_sha256": sha(m.labels_.astype(np.int32)),
           "products_centers_sha256": sha(m.cluster_centers_.astype(np.float32))}
    out = {"products_centers": m.cluster_centers_.astype(np.float32)}
    for name, n, k in (("users", 6040, 604), ("items", 3706, 371)):
        E = synth.svd_like(n, 64, seed=n)
        lab, cen = recsys.kmeans_cluster(E, n_clusters=k, seed=42, minibatch=True)
        out[f"ml1m_{name}_labels"] = lab.astype(np.int16)
        out[f"ml1m_{name}_centers"] = cen.astype(np.float32)
        rec[f"ml1m_{name}_input"] = f"gdd.synth.svd_like({n}, 64, seed={n})"
    rec["ml1m_call"] = "distill_recsys.kmeans_cluster(E, n_clusters=k, seed=42, minibatch=True)"
    np.savez_compressed(os.path.join(OUT, "golden_configs.npz"), **out)
    with open(os.path.join(OUT, "golden_configs.json"), "w") as f:
        json.dump(rec, f, indent=1)


def g9b_full_shapes():
    """k-means at the full config-3 and config-5 shapes, as hashes: MiniBatchKMeans(k=769,
    b=1000, random_state=15) on a 153,932 x 41 Reddit-train-shaped input (k > b/2: the reassignment's
    argsort branch can fire), and KMeans(k=196) on the full 2,449,029 x 47 products-shaped input after
    np.random.seed(15) (the agent's random_state=None call)."""
    import time
    from sklearn.cluster import KMeans, MiniBatchKMeans
    rec = {}
    t = time.time()
    X = synth.blobs(153932, 41, 769, seed=41)
    m = MiniBatchKMeans(n_clusters=769, random_state=15, batch_size=1000).fit(X)
    rec.update(reddit_input="gdd.synth.blobs(153932, 41, 769, seed=41)",
               reddit_estimator="MiniBatchKMeans(n_clusters=769, random_state=15, batch_size=1000)",
               reddit_n_steps=int(m.n_steps_), reddit_inertia=float(m.inertia_),
               reddit_labels_sha256=sha(m.labels_.astype(np.int32)),
               reddit_centers_sha256=sha(m.cluster_centers_.astype(np.float32)),
               reddit_seconds=time.time() - t)
    t = time.time()
    X = synth.blobs(2449029, 47, 196, seed=5)
    np.random.seed(15)
    m = KMeans(n_clusters=196).fit(X)
    rec.update(products_input="gdd.synth.blobs(2449029, 47, 196, seed=5)",
               products_estimator="np.random.seed(15); KMeans(n_clusters=196) (random_state=None)",
               products_n_iter=int(m.n_iter_), products_inertia=float(m.inertia_),
               products_labels_sha256=sha(m.labels_.astype(np.int32)),
               products_centers_sha256=sha(m.cluster_centers_.astype(np.float32)),
               products_seconds=time.time() - t)
    with open(os.path.join(OUT, "golden_full_shapes.json"), "w") as f:
        json.dump(rec, f, indent=1)


class _Args:
    pass


def g10_agent(agent_mod):
    import io
    import random
    import contextlib
    import torch
    sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
    from gdd import data as D
    from gdd.train_clustgdd_transduct import parser
    args = parser().parse_args(["--dataset", "cora", "--reduction_rate", "0.5", "--prop_num", "5",
                                "--postprop_num", "2", "--alpha", "0.8", "--predropout", "0.6",
                                "--sp_ratio", "0.4", "--preep", "80", "--postep", "200",
                                "--frcoe", "0.01", "--predcoe", "1.0"])
    random.seed(args.seed)
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    data = D.synthetic("cora", seed=args.seed, d=300)
    cap = {}
    orig_pc = agent_mod.ClustGDD.pretrained_clustering
    orig_tv = agent_mod.ClustGDD.test_with_val
    orig_km = agent_mod.KMeans

    class KMeansCap(orig_km):
        def fit(self, X, *a, **k):
            cap["kmeans_input"] = np.asarray(X, np.float32).copy()
            cap["np_state_key"] = np.random.get_state()[1].copy()
            cap["np_state_pos"] = np.int64(np.random.get_state()[2])
            return super().fit(X, *a, **k)

    def pc(self, data_):
        out = orig_pc(self, data_)
        cap["feat_syn_pre"] = out[0].detach().numpy()
        cap["labels_syn"] = out[1].numpy()
        cap["cluster_labels"] = out[2].numpy()
        return out

    runs = []

    def tv(self, i, verbose=True):
        if not runs:
            cap["torch_rng_state"] = torch.get_rng_state().numpy().copy()
        r = orig_tv(self, i, verbose)
        runs.append(r)
        return r

    agent_mod.KMeans = KMeansCap
    agent_mod.ClustGDD.pretrained_clustering = pc
    agent_mod.ClustGDD.test_with_val = tv
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.cuda.max_memory_allocated = lambda *a, **k: 0
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        agent = agent_mod.ClustGDD(data, args, device="cpu")
        agent.train()
    out = dict(cap)
    out.update(feat_syn=agent.feat_syn.detach().numpy(), adj_syn=agent.adj_syn.numpy(),
               labels_syn_final=agent.labels_syn.numpy(), runs=np.asarray(runs, np.float64))
    np.savez_compressed(os.path.join(OUT, "golden_agent.npz"), **out)
    with open(os.path.join(OUT, "golden_agent_stdout.txt"), "w") as f:
        f.write(buf.getvalue())


def g5_clustgdd(agent, dataset):
    """ClustGDD.pretrained_clustering on a small synthetic graph (device='cpu')."""
    import torch
    n, d, C = 600, 50, 5
    rng = np.random.default_rng(41)
    labels = rng.integers(0, C, n)
    mu = rng.standard_normal((C, d)) * 1.5
    feat = (mu[labels] + rng.standard_normal((n, d))).astype(np.float32)
    # a homophilous graph: most edges inside a class
    src = rng.integers(0, n, 3000)
    same = rng.random(3000) < 0.8
    dst = np.where(same, [rng.choice(np.where(labels == labels[s])[0]) for s in src],
                   rng.integers(0, n, 3000))
    keep = src != dst
    A = sp.coo_matrix((np.ones(keep.sum(), np.float32), (src[keep], dst[keep])), shape=(n, n))
    A = sp.csr_matrix(A + A.T)
    A.data[:] = 1.0
    A.sort_indices()
    idx_train, idx_val, idx_test = np.arange(0, 120), np.arange(120, 240), np.arange(240, n)

    data = types.SimpleNamespace(
        feat_full=feat, adj_full=A, labels_full=labels, idx_train=idx_train, idx_val=idx_val,
        idx_test=idx_test, feat_train=feat[idx_train], labels_train=labels[idx_train],
        labels_val=labels[idx_val], labels_test=labels[idx_test], nclass=C)
    args = _Args()
    args.reduction_rate, args.prop_num, args.alpha = 0.25, 5, 0.8
    args.hidden, args.predropout, args.prewd, args.prenlayers = 64, 0.6, 5e-4, 2
    args.prelr, args.preep, args.dataset, args.seed, args.cluster_minibatch = 0.01, 30, dataset, 15, 100

    captured = {}
    real_km, real_mb = agent.KMeans, agent.MiniBatchKMeans

    def capture(cls):
        class Wrapped(cls):
            def fit(self, X, *a, **kw):
                captured["X"] = np.array(X, copy=True)
                captured["rng_state"] = np.random.get_state()
                captured["params"] = {k: v for k, v in self.get_params().items()
                                      if k in ("n_clusters", "random_state", "batch_size", "n_init")}
                return super().fit(X, *a, **kw)
        return Wrapped

    agent.KMeans, agent.MiniBatchKMeans = capture(real_km), capture(real_mb)
    try:
        import random
        random.seed(15)
        np.random.seed(15)
        torch.manual_seed(15)
        a = agent.ClustGDD(data, args, device="cpu")
        res = a.pretrained_clustering(data)
    finally:
        agent.KMeans, agent.MiniBatchKMeans = real_km, real_mb
    feat_syn, labels_syn, cluster_labels, adj_norm = res[0], res[1], res[2], res[3]
    target_feat = res[7]
    r, c, v = coo_sorted(adj_norm)
    st = captured["rng_state"]
    rp, ci, vi = csr_arrays(A)
    out = {"rowptr": rp, "col": ci, "val": vi, "feat": feat, "T": np.int64(args.prop_num),
           "alpha": np.float64(args.alpha), "norm_row": r, "norm_col": c, "norm_val": v,
           "target_feat": target_feat.numpy(), "kmeans_X": captured["X"],
           "rng_key": st[1], "rng_pos": np.int64(st[2]), "rng_has_gauss": np.int64(st[3]),
           "rng_cached_gauss": np.float64(st[4]),
           "n_syn": np.int64(a.nnodes_syn), "feat_syn": feat_syn.numpy(),
           "labels_syn": labels_syn.numpy(), "cluster_labels": cluster_labels.numpy(),
           "kmeans_params": json.dumps({k: (v if not isinstance(v, np.integer) else int(v))
                                        for k, v in captured["params"].items()})}
    tag = "arxiv" if dataset == "ogbn-arxiv" else "cora"
    np.savez_compressed(os.path.join(OUT, f"golden_clustgdd_{tag}.npz"), **out)


def g6_condense(du, agent):
    """graph_sparse + graph_compress on a 500-node graph (C=5 classes, k=40 clusters), two label
    sets: every cluster populated, and cluster 17 empty (the reference's NaN row/column)."""
    import torch
    import utils_clustgdd as uc
    n, C, k, ratio = 500, 5, 40, 0.4
    A = synth.chung_lu(n, 8.0, 61)
    rp, ci, vi = csr_arrays(A)
    adj_norm = du.normalize_adj_tensor(du.sparse_mx_to_torch_sparse_tensor(sp.csr_matrix(A)),
                                       sparse=True)
    rng = np.random.default_rng(62)
    ebd = torch.from_numpy((rng.standard_normal((n, C)) * 2.0).astype(np.float32))
    r, c, v = coo_sorted(adj_norm)
    out = {"rowptr": rp, "col": ci, "val": vi, "norm_row": r, "norm_col": c, "norm_val": v,
           "ebd": ebd.numpy(), "ratio": np.float64(ratio), "k": np.int64(k)}
    a = adj_norm.coalesce()
    src, dst = a._indices()[0], a._indices()[1]
    er, rew = uc.attaw_ER_estimator(adj_norm, ebd, src, dst)
    out["er_attaw"] = er.numpy()
    out["reweighted_val"] = rew.coalesce()._values().numpy()
    out["er_vanilla"] = uc.ER_estimator(adj_norm, src, dst).numpy()
    for sp_type in ("attaw", "vanilla", "single"):
        gl = agent.ClustGDD.graph_sparse(None, adj_norm, ratio, ebd=ebd, sp_type=sp_type)
        out[f"{sp_type}_count"] = np.int64(len(gl))
        for q, g in enumerate(gl):
            gr, gc, gv = coo_sorted(g)
            out.update({f"{sp_type}{q}_row": gr, f"{sp_type}{q}_col": gc, f"{sp_type}{q}_val": gv})
    sparsed = agent.ClustGDD.graph_sparse(None, adj_norm, ratio, ebd=ebd, sp_type="attaw")
    lab_full = rng.permutation(np.arange(n) % k)
    lab_gap = lab_full.copy()
    lab_gap[lab_gap == 17] = 18
    for tag, lab in (("full", lab_full), ("gap", lab_gap)):
        cl, adj_syn = agent.ClustGDD.graph_compress(None, torch.from_numpy(lab), adj_norm, sparsed)
        out[f"{tag}_labels"] = lab.astype(np.int32)
        out[f"{tag}_adj_syn"] = adj_syn.to_dense().numpy()
        for q, g in enumerate(cl):
            out[f"{tag}_compressed{q}"] = g.to_dense().numpy()
    np.savez_compressed(os.path.join(OUT, "golden_condense.npz"), **out)


def g7_induct(dataset):
    """utils_graphsaint.DataGraphSAINT + clustgdd_agent_induct.ClustGDD.pretrained_clustering on a
    small synthetic GraphSAINT-format dataset (device='cpu')."""
    import random
    import tempfile
    import torch
    sys.path.insert(0, REF)
    import clustgdd_agent_induct as induct
    import utils_graphsaint as saint
    n, d, C = 900, 40, 5
    rng = np.random.default_rng(77 if dataset == "reddit" else 71)
    labels = rng.integers(0, C, n)
    mu = rng.standard_normal((C, d)) * 1.5
    feat = (mu[labels] + rng.standard_normal((n, d)) * 1.2 + 3.0).astype(np.float32)
    src = rng.integers(0, n, 5000)
    same = rng.random(5000) < 0.8
    dst = np.where(same, [rng.choice(np.where(labels == labels[s])[0]) for s in src],
                   rng.integers(0, n, 5000))
    keep = src != dst
    A = sp.coo_matrix((np.ones(keep.sum(), np.float32), (src[keep], dst[keep])), shape=(n, n))
    A = sp.csr_matrix(A + A.T)
    A.data[:] = 1.0
    A.sort_indices()
    role_of = rng.choice(3, n, p=[0.5, 0.2, 0.3])  # interleaved ascending role lists
    role = {"tr": np.where(role_of == 0)[0].tolist(), "va": np.where(role_of == 1)[0].tolist(),
            "te": np.where(role_of == 2)[0].tolist()}
    with tempfile.TemporaryDirectory() as tmp:
        base = os.path.join(tmp, "data", dataset)
        os.makedirs(base)
        sp.save_npz(os.path.join(base, "adj_full.npz"), A)
        np.save(os.path.join(base, "feats.npy"), feat)
        with open(os.path.join(base, "role.json"), "w") as f:
            json.dump(role, f)
        with open(os.path.join(base, "class_map.json"), "w") as f:
            json.dump({str(i): int(labels[i]) for i in range(n)}, f)
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            data = saint.DataGraphSAINT(dataset)
        finally:
            os.chdir(cwd)
    args = _Args()
    args.reduction_rate, args.prop_num, args.alpha = 0.2, 4, 0.8
    args.hidden, args.predropout, args.prewd, args.prenlayers = 64, 0.5, 5e-4, 2
    args.prelr, args.preep, args.dataset, args.seed, args.cluster_minibatch = 0.01, 30, dataset, 15, 100

    captured = {}
    real_km, real_mb = induct.KMeans, induct.MiniBatchKMeans

    def capture(cls):
        class Wrapped(cls):
            def fit(self, X, *a, **kw):
                captured["X"] = np.array(X, copy=True)
                captured["rng_state"] = np.random.get_state()
                captured["params"] = {k: v for k, v in self.get_params().items()
                                      if k in ("n_clusters", "random_state", "batch_size", "n_init")}
                return super().fit(X, *a, **kw)
        return Wrapped

    induct.KMeans, induct.MiniBatchKMeans = capture(real_km), capture(real_mb)
    try:
        random.seed(15)
        np.random.seed(15)
        torch.manual_seed(15)
        a = induct.ClustGDD(data, args, device="cpu")
        res = a.pretrained_clustering(data)
    finally:
        induct.KMeans, induct.MiniBatchKMeans = real_km, real_mb
    feat_syn, labels_syn, cluster_labels, target_train, adj_train_norm = res[:5]
    target_val = res[6]
    st = captured["rng_state"]
    out = {"T": np.int64(args.prop_num), "alpha": np.float64(args.alpha),
           "feat_raw": feat, "labels": labels.astype(np.int64),
           "idx_train": data.idx_train.astype(np.int64), "idx_val": data.idx_val.astype(np.int64),
           "idx_test": data.idx_test.astype(np.int64),
           "feat_full": np.asarray(data.feat_full), "target_train": target_train.numpy(),
           "target_val": target_val.numpy(), "kmeans_X": captured["X"],
           "rng_key": st[1], "rng_pos": np.int64(st[2]), "rng_has_gauss": np.int64(st[3]),
           "rng_cached_gauss": np.float64(st[4]),
           "n_syn": np.int64(a.nnodes_syn), "feat_syn": feat_syn.numpy(),
           "labels_syn": labels_syn.numpy(), "cluster_labels": cluster_labels.numpy(),
           "kmeans_params": json.dumps({k: (v if not isinstance(v, np.integer) else int(v))
                                        for k, v in captured["params"].items()})}
    rp, ci, vi = csr_arrays(A)
    out.update(rowptr=rp, col=ci, val=vi)
    for name in ("train", "val", "test"):
        sub = getattr(data, "adj_" + name).tocsr()
        out[f"sub_{name}_rowptr"], out[f"sub_{name}_col"], out[f"sub_{name}_val"] = csr_arrays(sub)
    r, c, v = coo_sorted(adj_train_norm)
    out.update(norm_train_row=r, norm_train_col=c, norm_train_val=v)
    np.savez_compressed(os.path.join(OUT, f"golden_clustgdd_induct_{dataset}.npz"), **out)


def _saint_files(tmp, dataset, n, d, C, seed):
    """A small GraphSAINT-format dataset (adj_full.npz, feats.npy, role.json, class_map.json) under
    tmp/data/<dataset>; returns the raw arrays."""
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, C, n)
    mu = rng.standard_normal((C, d)) * 0.4  # overlapping classes: accuracies well below 1
    feat = (mu[labels] + rng.standard_normal((n, d)) * 1.2 + 3.0).astype(np.float32)
    src = rng.integers(0, n, 6 * n)
    same = rng.random(6 * n) < 0.8
    dst = np.where(same, [rng.choice(np.where(labels == labels[s_])[0]) for s_ in src],
                   rng.integers(0, n, 6 * n))
    keep = src != dst
    A = sp.coo_matrix((np.ones(keep.sum(), np.float32), (src[keep], dst[keep])), shape=(n, n))
    A = sp.csr_matrix(A + A.T)
    A.data[:] = 1.0
    A.sort_indices()
    role_of = rng.choice(3, n, p=[0.5, 0.2, 0.3])
    role = {"tr": np.where(role_of == 0)[0].tolist(), "va": np.where(role_of == 1)[0].tolist(),
            "te": np.where(role_of == 2)[0].tolist()}
    base = os.path.join(tmp, "data", dataset)
    os.makedirs(base)
    sp.save_npz(os.path.join(base, "adj_full.npz"), A)
    np.save(os.path.join(base, "feats.npy"), feat)
    with open(os.path.join(base, "role.json"), "w") as f:
        json.dump(role, f)
    with open(os.path.join(base, "class_map.json"), "w") as f:
        json.dump({str(i): int(labels[i]) for i in range(n)}, f)
    return A, feat, labels, role


def g12_agent_induct(dataset):
    """The reference inductive agent (clustgdd_agent_induct.ClustGDD.train) end to end on the CPU on a
    small GraphSAINT-format dataset, with the flags of main_induct.sh's flickr lines (epochs cut):
    the k-means input and RNG state, the pre-refusion outputs, graph_refusion's inputs (dense
    compressed graphs) and torch RNG state, the refined features, the distilled graph, the torch RNG
    state before the GCN runs, the five [train, test] accuracies and stdout."""
    import contextlib
    import io
    import random
    import tempfile
    import torch
    sys.path.insert(0, REF)
    import clustgdd_agent_induct as induct
    import utils_graphsaint as saint
    from gdd.train_clustgdd_induct import parser
    argv = ["--dataset", dataset, "--reduction_rate", "0.05", "--prop_num", "2", "--postprop_num", "2",
            "--alpha", "0.8", "--predropout", "0.6", "--sp_ratio", "0.5", "--preep", "100", "--postep",
            "200", "--frcoe", "0.2", "--predcoe", "0.8", "--w1", "0.8", "--hidden", "64"]
    args = parser().parse_args(argv)
    with tempfile.TemporaryDirectory() as tmp:
        A, feat, labels, role = _saint_files(tmp, dataset, 900, 40, 5, 121 if dataset == "flickr" else 122)
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            data = saint.DataGraphSAINT(dataset)
        finally:
            os.chdir(cwd)
    cap = {}
    orig = {name: getattr(induct.ClustGDD, name) for name in
            ("pretrained_clustering", "graph_refusion", "test_with_val")}
    real_km, real_mb = induct.KMeans, induct.MiniBatchKMeans

    def capture(cls):
        class Wrapped(cls):
            def fit(self, X, *a, **kw):
                cap["kmeans_X"] = np.array(X, np.float32, copy=True)
                st = np.random.get_state()
                cap.update(rng_key=st[1], rng_pos=np.int64(st[2]), rng_has_gauss=np.int64(st[3]),
                           rng_cached_gauss=np.float64(st[4]))
                return super().fit(X, *a, **kw)
        return Wrapped

    def pc(self, data_):
        out = orig["pretrained_clustering"](self, data_)
        cap.update(feat_syn_pre=out[0].detach().numpy(), labels_syn=out[1].numpy(),
                   cluster_labels=out[2].numpy(), target_train=out[3].numpy(), target_val=out[6].numpy(),
                   logits_train=out[8].numpy())
        r, c, v = coo_sorted(out[4])
        cap.update(norm_train_row=r, norm_train_col=c, norm_train_val=v)
        return out

    def gr(self, ttrain, tval, ltrain, lval, feat_syn, graphs, label_syn):
        cap["refusion_rng_state"] = torch.get_rng_state().numpy().copy()
        cap["compressed_count"] = np.int64(len(graphs))
        for q, g in enumerate(graphs):
            cap[f"compressed{q}"] = g.to_dense().numpy()
        out = orig["graph_refusion"](self, ttrain, tval, ltrain, lval, feat_syn, graphs, label_syn)
        cap["feat_syn_refined"] = out.detach().numpy()
        return out

    runs = []

    def tv(self, i, verbose=True):
        if not runs:
            cap["torch_rng_state"] = torch.get_rng_state().numpy().copy()
        r = orig["test_with_val"](self, i, verbose)
        runs.append(r)
        return r

    induct.KMeans, induct.MiniBatchKMeans = capture(real_km), capture(real_mb)
    induct.ClustGDD.pretrained_clustering = pc
    induct.ClustGDD.graph_refusion = gr
    induct.ClustGDD.test_with_val = tv
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.cuda.max_memory_allocated = lambda *a, **k: 0
    buf = io.StringIO()
    try:
        random.seed(args.seed)
        np.random.seed(args.seed)
        torch.manual_seed(args.seed)
        with contextlib.redirect_stdout(buf):
            agent = induct.ClustGDD(data, args, device="cpu")
            ret = agent.train()
    finally:
        induct.KMeans, induct.MiniBatchKMeans = real_km, real_mb
        for name, f in orig.items():
            setattr(induct.ClustGDD, name, f)
    out = dict(cap)
    rp, ci, vi = csr_arrays(A)
    out.update(rowptr=rp, col=ci, val=vi, feat_raw=feat, labels=labels.astype(np.int64),
               idx_train=np.asarray(role["tr"], np.int64), idx_val=np.asarray(role["va"], np.int64),
               idx_test=np.asarray(role["te"], np.int64), feat_full=np.asarray(data.feat_full),
               n_syn=np.int64(agent.nnodes_syn), feat_syn=agent.feat_syn.detach().numpy(),
               adj_syn=agent.adj_syn.numpy(), labels_syn_final=agent.labels_syn.numpy(),
               adj_syn_raw=ret[1].to_dense().numpy(), runs=np.asarray(runs, np.float64),
               argv=json.dumps(argv))
    np.savez_compressed(os.path.join(OUT, f"golden_agent_induct_{dataset}.npz"), **out)
    with open(os.path.join(OUT, f"golden_agent_induct_{dataset}_stdout.txt"), "w") as f:
        f.write(buf.getvalue())


def g8_recsys(recsys):
    """The recommender's condensation and LightGCN refinement model (device='cpu')."""
    import torch
    rng = np.random.default_rng(81)
    nu, ni, E = 900, 600, 7000
    train_u = rng.integers(0, nu, E).astype(np.int64)
    train_i = (rng.zipf(1.6, E) % ni).astype(np.int64)  # popular items: many duplicate pairs
    num_cu, num_ci = 90, 60
    u2cu = rng.integers(0, num_cu - 3, nu).astype(np.int64)  # the last 3 super-users stay empty
    i2ci = rng.integers(0, num_ci, ni).astype(np.int64)
    C = recsys.build_condensed_bipartite(train_u, train_i, u2cu, i2ci, num_cu, num_ci)
    edge_index, w0 = recsys.condensed_csr_to_edge_index(C, device=torch.device("cpu"))
    torch.manual_seed(7)
    model = recsys.LightGCNCondensed(num_cu=num_cu, num_ci=num_ci, dim=32, num_layers=3,
                                     edge_index=edge_index, edge_weight_init=w0,
                                     device=torch.device("cpu"))
    with torch.no_grad():  # non-trivial deltas and edge logits
        model.user_delta.copy_(torch.randn(num_cu, 32) * 0.05)
        model.item_delta.copy_(torch.randn(num_ci, 32) * 0.05)
        model.edge_logit.add_(torch.randn(edge_index.shape[1]) * 0.3)
    params = {k: v.detach().clone().numpy() for k, v in model.named_parameters()}
    u_out, i_out = model.propagate()
    bu = torch.from_numpy(rng.integers(0, num_cu, 256).astype(np.int64))
    bp = torch.from_numpy(rng.integers(0, num_ci, 256).astype(np.int64))
    bn = torch.from_numpy(rng.integers(0, num_ci, 256).astype(np.int64))
    loss = model.bpr_loss(bu, bp, bn, reg_lambda=1e-4)
    loss.backward()
    out = {"train_u": train_u, "train_i": train_i, "u2cu": u2cu, "i2ci": i2ci,
           "num_cu": np.int64(num_cu), "num_ci": np.int64(num_ci),
           "C_indptr": C.indptr.astype(np.int64), "C_indices": C.indices.astype(np.int64),
           "C_data": C.data.astype(np.float32), "edge_index": edge_index.numpy(), "w0": w0.numpy(),
           "u_out": u_out.detach().numpy(), "i_out": i_out.detach().numpy(),
           "bpr_u": bu.numpy(), "bpr_pos": bp.numpy(), "bpr_neg": bn.numpy(),
           "loss": np.float64(loss.item()), "dim": np.int64(32), "layers": np.int64(3)}
    for k, v in params.items():
        out["param_" + k.replace(".", "_")] = v
    for k, v in model.named_parameters():
        out["grad_" + k.replace(".", "_")] = v.grad.detach().numpy()
    np.savez_compressed(os.path.join(OUT, "golden_recsys.npz"), **out)


def g11_refine(recsys):
    """The recommender's refinement loop (distill_recsys.py:217-272 sampler, :446-497 recall, :504-764
    main on a small Rankformer-format dataset, device='cpu')."""
    import contextlib
    import io
    import tempfile
    import torch
    out = {}
    # (a) the BPR triplet sampler on condensed graphs with empty rows, a full row and tiny item sets
    rng = np.random.default_rng(111)
    cases = []
    for ci, (nu, ni, dens, batch, seed) in enumerate([(60, 40, 0.2, 512, 42), (25, 5, 0.5, 300, 7),
                                                       (30, 3, 0.9, 200, 3)]):
        M = (rng.random((nu, ni)) < dens).astype(np.float32)
        M[1] = 0.0            # a super-user without positives
        M[2] = 1.0            # a super-user whose every item is positive
        C = sp.csr_matrix(M)
        pos_lists = recsys._csr_row_to_set_list(C)
        r = np.random.RandomState(seed)
        u, p, n = recsys.sample_bpr_triplets_from_condensed(pos_lists, ni, batch, r)
        st = r.get_state(legacy=True)
        out[f"s{ci}_indptr"], out[f"s{ci}_indices"] = C.indptr.astype(np.int64), C.indices.astype(np.int64)
        out[f"s{ci}_meta"] = np.array([nu, ni, batch, seed], np.int64)
        out[f"s{ci}_u"], out[f"s{ci}_pos"], out[f"s{ci}_neg"] = u, p, n
        out[f"s{ci}_key"], out[f"s{ci}_statepos"] = st[1].astype(np.uint32), np.int64(st[2])
        cases.append(ci)
    out["sampler_cases"] = np.array(cases, np.int64)
    # (b) recall_at_k: continuous embeddings (no ties) and cluster-shared embeddings (ties)
    for tag, shared in (("r0", False), ("r1", True)):
        nu, ni, d = 400, 300, 16
        ue = rng.standard_normal((nu, d)).astype(np.float32)
        ie = rng.standard_normal((ni, d)).astype(np.float32)
        if shared:
            ie = rng.standard_normal((30, d)).astype(np.float32)[rng.integers(0, 30, ni)]
        tr_u, tr_i = rng.integers(0, nu, 3000), rng.integers(0, ni, 3000)
        te_u, te_i = rng.integers(0, nu, 900), rng.integers(0, ni, 900)
        Rtr = sp.coo_matrix((np.ones(3000, np.float32), (tr_u, tr_i)), shape=(nu, ni)).tocsr()
        rec = recsys.recall_at_k(torch.from_numpy(ue), torch.from_numpy(ie), Rtr, te_u, te_i, 20,
                                 torch.device("cpu"), max_users=250)
        out.update({f"{tag}_ue": ue, f"{tag}_ie": ie, f"{tag}_tr_u": tr_u, f"{tag}_tr_i": tr_i,
                    f"{tag}_te_u": te_u, f"{tag}_te_i": te_i, f"{tag}_recall": np.float64(rec)})
    # (c) main() end to end on a small synthetic dataset (SVD embeddings captured: ARPACK's start
    # vector is not seeded by --seed)
    nu, ni = 600, 400
    users = rng.integers(0, nu, 9000)
    items = (rng.zipf(1.5, 9000) % ni)
    perm = rng.permutation(9000)
    tr, va, te = perm[:7000], perm[7000:8000], perm[8000:]
    argv = ["--dataset", "synth", "--reduction_rate", "0.1", "--svd_dim", "16", "--embed_dim", "16",
            "--lgn_layers", "2", "--refine_epochs", "6", "--batch_size", "256", "--log_every", "2",
            "--device", "cpu", "--eval_topk", "20", "--seed", "42"]
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "synth"))
        for name, idx in (("train", tr), ("valid", va), ("test", te)):
            np.savetxt(os.path.join(tmp, "synth", f"{name}.txt"), np.stack([users[idx], items[idx]], 1), fmt="%d")
        captured = {}
        orig_svd = recsys.compute_svd_embeddings

        def svd_capture(*a, **k):
            captured["emb"] = orig_svd(*a, **k)
            return captured["emb"]
        recsys.compute_svd_embeddings = svd_capture
        old_argv, cwd = sys.argv, os.getcwd()
        buf = io.StringIO()
        try:
            sys.argv = ["distill_recsys.py", "--data_dir", tmp] + argv
            os.chdir(tmp)
            with contextlib.redirect_stdout(buf):
                recsys.main()
            art = np.load(os.path.join(tmp, "ClustGDD", "distilled_recsys", "synth", "condensed_graph.npz"))
            out.update({"e2e_cu": art["cu"], "e2e_ci": art["ci"], "e2e_w": art["w"]})
            out["e2e_u2cu"] = np.load(os.path.join(tmp, "ClustGDD", "distilled_recsys", "synth", "u2cu.npy"))
            out["e2e_i2ci"] = np.load(os.path.join(tmp, "ClustGDD", "distilled_recsys", "synth", "i2ci.npy"))
        finally:
            sys.argv = old_argv
            os.chdir(cwd)
            recsys.compute_svd_embeddings = orig_svd
    out["e2e_users"], out["e2e_items"] = users, items
    out["e2e_split"] = np.stack([np.isin(np.arange(9000), tr), np.isin(np.arange(9000), va)], 0)
    out["e2e_user_emb"], out["e2e_item_emb"] = captured["emb"]
    np.savez_compressed(os.path.join(OUT, "golden_refine.npz"), **out)
    with open(os.path.join(OUT, "golden_refine_stdout.txt"), "w") as f:
        f.write(" ".join(argv) + "\n" + buf.getvalue())


def g6r_alidisplay(recsys):
    """distill_recsys.main() on the real Ali-Display data the reference ships
    (Rankformer/data/Ali-Display): a short refine (20 epochs, logged every 5) with
    stdout and artefacts, and the default 500-epoch run's stdout (the Recall@20 trajectory). The
    three split files are stored as integer arrays, the SVD embeddings as captured (svds draws its
    start vector from numpy's global generator; BLAS orders make its last bits platform-dependent)."""
    import contextlib
    import io
    import tempfile
    data_dir = "/root/reference/Rankformer/data"
    out = {}
    for split in ("train", "valid", "test"):
        a = np.loadtxt(os.path.join(data_dir, "Ali-Display", f"{split}.txt"), dtype=np.int64).reshape(-1, 2)
        out[f"{split}_u"], out[f"{split}_i"] = a[:, 0].astype(np.int32), a[:, 1].astype(np.int32)
    embs = []
    orig_svd = recsys.compute_svd_embeddings

    def svd_capture(*a, **k):
        embs.append(orig_svd(*a, **k))
        return embs[-1]
    recsys.compute_svd_embeddings = svd_capture
    runs = {"short": ["--refine_epochs", "20", "--log_every", "5"], "full": []}
    stdout = {}
    old_argv, cwd = sys.argv, os.getcwd()
    try:
        for tag, extra in runs.items():
            with tempfile.TemporaryDirectory() as tmp:
                argv = ["--data_dir", data_dir, "--dataset", "Ali-Display", "--device", "cpu"] + extra
                sys.argv = ["distill_recsys.py"] + argv
                os.chdir(tmp)
                buf = io.StringIO()
                with contextlib.redirect_stdout(buf):
                    recsys.main()
                stdout[tag] = " ".join(argv[2:]) + "\n" + buf.getvalue()
                if tag == "short":
                    base = os.path.join(tmp, "ClustGDD", "distilled_recsys", "Ali-Display")
                    art = np.load(os.path.join(base, "condensed_graph.npz"))
                    out.update({"cu": art["cu"], "ci": art["ci"], "w": art["w"],
                                "u2cu": np.load(os.path.join(base, "u2cu.npy")),
                                "i2ci": np.load(os.path.join(base, "i2ci.npy"))})
                os.chdir(cwd)
    finally:
        sys.argv = old_argv
        os.chdir(cwd)
        recsys.compute_svd_embeddings = orig_svd
    assert all(np.array_equal(embs[0][j], e[j]) for e in embs for j in range(2)), "svds not repeatable"
    out["user_emb"], out["item_emb"] = embs[0]
    np.savez_compressed(os.path.join(OUT, "golden_alidisplay.npz"), **out)
    for tag, text in stdout.items():
        with open(os.path.join(OUT, f"golden_alidisplay_{tag}_stdout.txt"), "w") as f:
            f.write(text)


def main():
    from threadpoolctl import threadpool_limits
    import sklearn
    import scipy
    import torch
    os.makedirs(OUT, exist_ok=True)
    du, agent, recsys = import_reference()
    which = set(sys.argv[1:]) or {"G1", "G2", "G3", "G3b", "G5", "G6", "G7", "G8", "G9"}
    with threadpool_limits(limits=1):
        if "G1" in which:
            g1_normalize(du)
        if "G2" in which:
            g2_propagate(du)
        if "G3" in which:
            g3_kmeans(recsys)
        if "G3b" in which:
            g3b_arxiv()
        if "G5" in which:
            g5_clustgdd(agent, "cora")
            g5_clustgdd(agent, "ogbn-arxiv")
        if "G6" in which:
            g6_condense(du, agent)
        if "G8" in which:
            g8_recsys(recsys)
        if "G9" in which:
            g9_configs(recsys)
        if "G9b" in which:
            g9b_full_shapes()
        if "G6r" in which:
            torch.set_num_threads(1)
            g6r_alidisplay(recsys)
        if "G11" in which:
            torch.set_num_threads(1)
            g11_refine(recsys)
        if "G10" in which:  # last: it patches torch.Tensor.cuda for its own run
            torch.set_num_threads(1)
            g10_agent(agent)
        if "G7" in which:
            g7_induct("flickr")
            g7_induct("reddit")
        if "G12" in which:  # patches torch.Tensor.cuda for its own run
            torch.set_num_threads(1)
            g12_agent_induct("flickr")
            g12_agent_induct("reddit")
    with open(os.path.join(OUT, "VERSIONS.json"), "w") as f:
        json.dump({"scikit-learn": sklearn.__version__, "numpy": np.__version__,
                   "scipy": scipy.__version__, "torch": torch.__version__,
                   "threads": 1, "reference": "/root/reference snapshot 2026-04-03"}, f, indent=1)
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
