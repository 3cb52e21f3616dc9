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
