"""The gdd-backed ClustGDD agent (gdd.agent, the drop-in for clustgdd_agent_transduct.py) on the
GPU against the reference's own run (fixture G10, the reference agent on the CPU).

* the clustering stage from the reference's k-means input (its numpy RNG state restored): the
  cluster labels and labels_syn bit for bit, the pre-refusion feat_syn within the propagation
  tolerance (our propagation order is the canonical one, the reference's is torch's);
* the whole agent (pretrained_clustering -> graph_sparse -> graph_compress -> graph_refusion ->
  5 x test_with_val) on the GPU prints the reference's lines, and its Train/Test Mean Accuracy is
  the reference's within 0.03 (the MLP/GCN train on another device's RNG streams, SURVEY App. A.6,
  so the accuracies agree statistically, not bit for bit; the CPU test test_agent_cpu.py pins the
  evaluator itself exactly).
"""
import contextlib
import io
import random

import numpy as np
import pytest
import torch

from golden_util import MEAN_ATOL, MEAN_RTOL, load

pytestmark = pytest.mark.gpu

import gdd  # noqa: E402
from gdd import data as D  # noqa: E402
from gdd.train_clustgdd_transduct import parser  # noqa: E402

ARGS = ["--dataset", "cora", "--reduction_rate", "0.5", "--prop_num", "5", "--postprop_num", "2",
        "--alpha", "0.8", "--predropout", "0.6", "--sp_ratio", "0.4", "--preep", "80",
        "--postep", "200", "--frcoe", "0.01", "--predcoe", "1.0"]


def test_clustering_stage_matches_reference_agent():
    z = load("golden_agent.npz")
    data = D.synthetic("cora", seed=15, d=300)
    np.random.set_state(("MT19937", z["np_state_key"], int(z["np_state_pos"]), 0, 0.0))
    km = gdd.KMeans(n_clusters=70).fit(z["kmeans_input"])
    assert np.array_equal(km.labels_, z["cluster_labels"])
    assert np.array_equal(gdd.argmax_rows(km.cluster_centers_device_).cpu().numpy(), z["labels_syn"])
    g = gdd.normalize_adj(gdd.to_csr(data.adj_full, device="cuda"))
    target, _ = gdd.propagate(g, torch.from_numpy(data.feat_full).cuda(), 5, 0.8)
    fs, _ = gdd.cluster_mean(target, km.labels_device_, 70)
    np.testing.assert_allclose(fs.cpu().numpy(), z["feat_syn_pre"], rtol=MEAN_RTOL, atol=MEAN_ATOL)


def test_agent_end_to_end_accuracy_and_stdout():
    z = load("golden_agent.npz")
    from gdd.agent import ClustGDD
    args = parser().parse_args(ARGS)
    random.seed(args.seed)
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    torch.cuda.manual_seed(args.seed)
    data = D.synthetic("cora", seed=args.seed, d=300)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        agent = ClustGDD(data, args, device="cuda:0")
        agent.train()
    out = buf.getvalue()
    for line in ("adj_syn: (1354, 1354) feat_syn: (1354, 300)"[:8], "MLP pretrain, train set results:",
                 "MLP pretrain, test set results:", "finish clustering", "Train/Test Mean Accuracy:",
                 "The pretraining time is", "The refinement time is", "Total time is",
                 "max memory allocation:"):
        assert line in out, line
    assert agent.feat_syn.shape == (70, 300) and agent.adj_syn.shape == (70, 70)
    ref = z["runs"].mean(0)
    got = agent.results.mean(0)
    assert abs(got[1] - ref[1]) <= 0.03, (got, ref)
    assert abs(got[0] - ref[0]) <= 0.05, (got, ref)


# ---- the inductive agent (gdd.agent_induct, drop-in for clustgdd_agent_induct.py), fixture G12 ----
def _saint_dir(z, tmp, tag):
    """Writes the fixture's dataset in the GraphSAINT format (the reference read the same files)."""
    import json
    import os
    import scipy.sparse as sp
    n = z["feat_raw"].shape[0]
    base = os.path.join(str(tmp), tag)
    os.makedirs(base)
    sp.save_npz(os.path.join(base, "adj_full.npz"), sp.csr_matrix((z["val"], z["col"], z["rowptr"]),
                                                                  shape=(n, n)))
    np.save(os.path.join(base, "feats.npy"), z["feat_raw"])
    with open(os.path.join(base, "role.json"), "w") as f:
        json.dump({"tr": z["idx_train"].tolist(), "va": z["idx_val"].tolist(), "te": z["idx_test"].tolist()}, f)
    with open(os.path.join(base, "class_map.json"), "w") as f:
        json.dump({str(i): int(v) for i, v in enumerate(z["labels"])}, f)
    return base


class _FixedLogits:
    """Stands in for MLP_Induct in the clustering stage: the reference's own train logits."""
    logits = None

    def __init__(self, *a, **k):
        pass

    def to(self, dev):
        return self

    def fit_with_val(self, *a, **k):
        pass

    def eval(self):
        pass

    def predict(self, x, mode="t"):  # the train logits; zeros for the test role (printed only)
        out = torch.from_numpy(self.logits).to(x.device)
        if out.shape[0] != x.shape[0]:
            out = torch.zeros((x.shape[0], out.shape[1]), device=x.device)
        return torch.log_softmax(out, 1), out


@pytest.mark.parametrize("tag", ["flickr", "reddit"])
def test_induct_clustering_stage_matches_reference_agent(tmp_path, monkeypatch, tag):
    """load_graphsaint + the inductive pretrained_clustering on the GPU from the reference's train
    logits (numpy RNG restored for KMeans): cluster labels and labels_syn bit for bit, the train
    targets and feat_syn within the propagation tolerance, the normalised train graph exact."""
    import json
    from gdd import agent_induct, pipeline
    from gdd.train_clustgdd_induct import parser as ip
    z = load(f"golden_agent_induct_{tag}.npz")
    args = ip().parse_args(json.loads(str(z["argv"])))
    data = pipeline.load_graphsaint(_saint_dir(z, tmp_path, tag), tag, device="cuda")
    np.testing.assert_array_equal(data.feat_full.cpu().numpy().view(np.uint32),
                                  np.ascontiguousarray(z["feat_full"], np.float32).view(np.uint32))
    _FixedLogits.logits = z["logits_train"]
    monkeypatch.setattr(agent_induct, "MLP_Induct", _FixedLogits)
    np.random.set_state(("MT19937", z["rng_key"], int(z["rng_pos"]), int(z["rng_has_gauss"]),
                         float(z["rng_cached_gauss"])))
    with contextlib.redirect_stdout(io.StringIO()):
        agent = agent_induct.ClustGDD(data, args, device="cuda")
        out = agent.pretrained_clustering(data)
    feat_syn, labels_syn, cluster_labels, target_train, adj_train_norm = out[:5]
    assert np.array_equal(cluster_labels.cpu().numpy(), z["cluster_labels"])
    assert np.array_equal(labels_syn.cpu().numpy(), z["labels_syn"])
    np.testing.assert_allclose(target_train.cpu().numpy(), z["target_train"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out[6].cpu().numpy(), z["target_val"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(feat_syn.cpu().numpy(), z["feat_syn_pre"], rtol=MEAN_RTOL, atol=MEAN_ATOL)
    sc = adj_train_norm.to_scipy().tocoo()
    o = np.lexsort((sc.col, sc.row))
    assert np.array_equal(sc.row[o], z["norm_train_row"]) and np.array_equal(sc.col[o], z["norm_train_col"])
    assert np.array_equal(sc.data[o].astype(np.float32).view(np.uint32), z["norm_train_val"].view(np.uint32))


@pytest.mark.parametrize("tag", ["flickr", "reddit"])
def test_induct_agent_end_to_end(tmp_path, tag):
    """gdd.train_clustgdd_induct with the fixture's flags on the GraphSAINT files: the reference's
    stdout lines, train() returning (adj_train_norm, adj_syn, feat_syn, labels_syn), and the
    Train/Test Mean Accuracy within 0.05 of the reference's CPU run (the MLPs and the GCN train on
    the GPU's RNG streams: statistically equal, not bit for bit — the CPU test pins the torch stages
    exactly)."""
    import json
    from gdd import train_clustgdd_induct as T
    z = load(f"golden_agent_induct_{tag}.npz")
    argv = json.loads(str(z["argv"])) + ["--data_dir", _saint_dir(z, tmp_path, tag)]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        agent, (adj_train_norm, adj_syn, feat_syn, labels_syn) = T.main(argv)
    out = buf.getvalue()
    ref = open(__import__("golden_util").GOLDEN + f"/golden_agent_induct_{tag}_stdout.txt").read()
    for line in ref.splitlines():
        key = line.split(":")[0].split(",")[0].split(" is ")[0]
        assert key in out, key
    k = int(z["n_syn"])
    assert feat_syn.shape == (k, z["feat_raw"].shape[1]) and adj_syn.shape == (k, k) and adj_syn.is_sparse
    assert labels_syn.shape == (k,) and adj_train_norm.n == z["idx_train"].shape[0]
    got, want = agent.results.mean(0), z["runs"].mean(0)
    assert abs(got[1] - want[1]) <= 0.05 and abs(got[0] - want[0]) <= 0.05, (got, want)
