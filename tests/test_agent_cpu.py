"""The downstream metric's machinery ("Train/Test Mean Accuracy" of 5 GCN runs on the
distilled graph, clustgdd_agent_transduct.py:349-425) against the reference's own run (fixture
G10: the reference ClustGDD agent end to end on the CPU, one thread).

Given the reference's distilled graph (feat_syn, the normalised dense adj_syn, labels_syn) and its
torch RNG state at the start of the evaluation, gdd.agent.ClustGDD.test_with_val (gdd.models.GCN:
the same parameters, initialisation order, dropout draws, Adam restarts and best-validation rule)
must reproduce the five [train, test] accuracies exactly. CPU only, no GPU or libgdd needed.
"""
import types

import numpy as np
import torch

from golden_util import load


def test_gcn_evaluation_reproduces_reference_accuracies():
    z = load("golden_agent.npz")
    from gdd import data as D
    from gdd.agent import ClustGDD
    from gdd.train_clustgdd_transduct import parser
    args = parser().parse_args(["--dataset", "cora", "--reduction_rate", "0.5"])
    torch.set_num_threads(1)
    data = D.synthetic("cora", seed=15, d=300)
    agent = ClustGDD.__new__(ClustGDD)  # no distillation: the reference's distilled graph is given
    agent.data, agent.args, agent.device = data, args, "cpu"
    agent.feat_syn = torch.from_numpy(z["feat_syn"])
    agent.adj_syn = torch.from_numpy(z["adj_syn"])
    agent.labels_syn = torch.from_numpy(z["labels_syn_final"])
    torch.set_rng_state(torch.from_numpy(z["torch_rng_state"]))
    runs = np.array([agent.test_with_val(i, verbose=False) for i in range(5)])
    assert np.array_equal(runs, z["runs"]), (runs, z["runs"])
    mean = runs.mean(0)
    assert mean[1] > 0.5  # learnable synthetic data: far above chance (7 classes)


def test_synthetic_dataset_matches_transd2ind_layout():
    from gdd import data as D
    d = D.synthetic("cora", seed=3, d=64)
    assert d.nclass == 7 and d.feat_full.shape == (2708, 64)
    assert len(d.idx_train) == 140 and len(d.idx_val) == 500 and len(d.idx_test) == 1000
    assert not set(d.idx_train) & set(d.idx_val) and not set(d.idx_val) & set(d.idx_test)
    assert d.adj_train.shape == (140, 140) and np.array_equal(d.labels_train, d.labels_full[d.idx_train])
    A = d.adj_full
    assert (A != A.T).nnz == 0 and A.diagonal().sum() == 0
    same = (d.labels_full[A.nonzero()[0]] == d.labels_full[A.nonzero()[1]]).mean()
    assert same > 0.6  # homophilous
