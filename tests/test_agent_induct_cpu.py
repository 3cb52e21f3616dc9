"""The inductive drop-in agent's torch stages against the reference's own run (fixture G12: the
reference clustgdd_agent_induct.ClustGDD.train end to end on the CPU, one thread, on small
GraphSAINT-format datasets — 'flickr' clusters with KMeans, 'reddit' with MiniBatchKMeans).

Given the reference's inputs to each stage and its torch RNG state there, gdd.agent_induct.ClustGDD
must reproduce, exactly:
* graph_refusion (induct:276-372): the refined synthetic features (learnable reweight matrices,
  three Adam optimisers with the half-way restart, best-validation refine) and its stdout lines;
* test_with_val x 5 (induct:374-421): the five [train, test] accuracies of the GCN trained on the
  distilled graph, validated on the val sub-graph and scored on the train / test sub-graphs.
CPU only (the libgdd stages are covered by tests/test_gpu_agent.py on the same fixture).
"""
import contextlib
import io
import json
import types

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from golden_util import GOLDEN, load


def _agent(z, tag):
    from gdd.agent_induct import ClustGDD
    from gdd.train_clustgdd_induct import parser
    args = parser().parse_args(json.loads(str(z["argv"])))
    agent = ClustGDD.__new__(ClustGDD)
    agent.args, agent.device = args, "cpu"
    n = z["feat_raw"].shape[0]
    A = sp.csr_matrix((z["val"], z["col"], z["rowptr"]), shape=(n, n))
    labels = z["labels"]
    data = types.SimpleNamespace(nclass=int(labels.max()) + 1, feat_full=z["feat_full"], adj_full=A,
                                 labels_full=labels)
    for role in ("train", "val", "test"):
        idx = z["idx_" + role]
        setattr(data, "idx_" + role, idx)
        setattr(data, "feat_" + role, z["feat_full"][idx])
        setattr(data, "adj_" + role, A[np.ix_(idx, idx)])
        setattr(data, "labels_" + role, labels[idx])
    agent.data = data
    return agent


@pytest.mark.parametrize("tag", ["flickr", "reddit"])
def test_graph_refusion_reproduces_reference(tag):
    z = load(f"golden_agent_induct_{tag}.npz")
    torch.set_num_threads(1)
    agent = _agent(z, tag)
    d = agent.data
    graphs = [torch.from_numpy(z[f"compressed{q}"]) for q in range(int(z["compressed_count"]))]
    torch.set_rng_state(torch.from_numpy(z["refusion_rng_state"]))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        out = agent.graph_refusion(torch.from_numpy(z["target_train"]), torch.from_numpy(z["target_val"]),
                                   torch.LongTensor(d.labels_train), torch.LongTensor(d.labels_val),
                                   torch.from_numpy(z["feat_syn_pre"]), graphs,
                                   torch.from_numpy(z["labels_syn"]))
    assert np.array_equal(out.detach().numpy().view(np.uint32), z["feat_syn_refined"].view(np.uint32))
    ref = open(f"{GOLDEN}/golden_agent_induct_{tag}_stdout.txt").read().splitlines()
    lo = ref.index("start post training") + 1
    hi = next(i for i in range(lo, len(ref)) if ref[i].startswith("Train set results"))
    assert buf.getvalue().splitlines() == ref[lo:hi]


@pytest.mark.parametrize("tag", ["flickr", "reddit"])
def test_gcn_evaluation_reproduces_reference_accuracies(tag):
    z = load(f"golden_agent_induct_{tag}.npz")
    torch.set_num_threads(1)
    agent = _agent(z, tag)
    agent.feat_syn = torch.from_numpy(z["feat_syn"])
    agent.adj_syn = torch.from_numpy(z["adj_syn"])
    agent.labels_syn = torch.from_numpy(z["labels_syn_final"])
    torch.set_rng_state(torch.from_numpy(z["torch_rng_state"]))
    runs = np.array([agent.test_with_val(i, verbose=False) for i in range(5)])
    assert np.array_equal(runs, z["runs"]), (runs, z["runs"])


def test_induct_cli_flags_match_reference_defaults():
    from gdd.train_clustgdd_induct import parser as ind
    from gdd.train_clustgdd_transduct import parser as tr
    a, b = ind().parse_args([]), tr().parse_args([])
    assert a.sp_ratio == 1.0 and b.sp_ratio == 0.05 and a.epochs == 2000 and not hasattr(b, "epochs")
    assert {k for k in vars(a)} - {k for k in vars(b)} == {"epochs"}
