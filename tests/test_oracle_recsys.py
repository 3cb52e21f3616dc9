"""CPU: the recommender condensation oracle against the reference's own output (G8), and the
artefact writer's formats (distill_recsys.py:736-764)."""
import os

import numpy as np
import torch

from golden_util import load
from oracle import recsys as R


def test_condense_oracle_vs_reference():
    z = load("golden_recsys.npz")
    rp, c, v = R.build_condensed_bipartite(z["train_u"], z["train_i"], z["u2cu"], z["i2ci"],
                                           int(z["num_cu"]), int(z["num_ci"]))
    assert np.array_equal(rp, z["C_indptr"]) and np.array_equal(c, z["C_indices"])
    assert np.array_equal(v, z["C_data"])
    # condensed_csr_to_edge_index: CSR order
    rows = np.repeat(np.arange(int(z["num_cu"])), np.diff(rp))
    assert np.array_equal(z["edge_index"], np.vstack([rows, c]))
    assert rp[-1] == rp[-4]  # the three empty super-users


def test_save_distilled_formats(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "graph-distillation-for-recommendation_amd"))
    from gdd import recsys
    z = load("golden_recsys.npz")
    ei = torch.from_numpy(z["edge_index"])
    m = recsys.LightGCNCondensed(int(z["num_cu"]), int(z["num_ci"]), 8, 2, ei, torch.from_numpy(z["w0"]),
                                 device=torch.device("cpu"))
    recsys.save_distilled(str(tmp_path), m, z["u2cu"], z["i2ci"], int(z["num_cu"]), int(z["num_ci"]))
    g = np.load(tmp_path / "condensed_graph.npz")
    assert sorted(g.files) == ["ci", "cu", "num_ci", "num_cu", "w"]
    assert g["cu"].dtype == np.int64 and g["ci"].dtype == np.int64 and g["w"].dtype == np.float32
    assert int(g["num_cu"]) == int(z["num_cu"]) and g["num_cu"].dtype == np.int64
    assert np.array_equal(g["cu"], z["edge_index"][0])
    np.testing.assert_allclose(g["w"], np.maximum(z["w0"], 1e-6), rtol=1e-5)  # softplus(inv_softplus(w))
    u2 = np.load(tmp_path / "u2cu.npy")
    assert u2.dtype == np.int64 and np.array_equal(u2, z["u2cu"])
    emb = torch.load(tmp_path / "condensed_embeddings.pt", weights_only=True)
    assert sorted(emb) == ["item_delta", "item_emb", "user_delta", "user_emb"]
    assert emb["user_emb"].shape == (int(z["num_cu"]), 8)


# ---- the refinement loop's helpers (G11: the reference's own sampler, recall_at_k and main()) ----
def _sampler_case(z, c):
    nu, ni, batch, seed = (int(v) for v in z[f"s{c}_meta"])
    ptr, idx = z[f"s{c}_indptr"], z[f"s{c}_indices"]
    rows = [idx[ptr[r]:ptr[r + 1]] for r in range(nu)]
    return rows, ptr, idx, nu, ni, batch, seed


def test_bpr_sampler_oracle_vs_reference():
    z = load("golden_refine.npz")
    for c in z["sampler_cases"]:
        rows, _, _, nu, ni, batch, seed = _sampler_case(z, c)
        rs = np.random.RandomState(seed)
        u, p, n = R.bpr_triplets(rows, ni, batch, rs)
        assert np.array_equal(u, z[f"s{c}_u"]) and np.array_equal(p, z[f"s{c}_pos"])
        assert np.array_equal(n, z[f"s{c}_neg"])
        st = rs.get_state(legacy=True)
        assert np.array_equal(st[1], z[f"s{c}_key"]) and st[2] == int(z[f"s{c}_statepos"])


def _gdd():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "graph-distillation-for-recommendation_amd"))
    from gdd import recsys
    return recsys


def test_native_bpr_sampler_vs_reference():
    # host-only native code in libgdd (gdd_bpr_sample): no device needed
    recsys = _gdd()
    z = load("golden_refine.npz")
    for c in z["sampler_cases"]:
        rows, ptr, idx, nu, ni, batch, seed = _sampler_case(z, c)
        pl = recsys.PositiveLists(ptr, idx)
        rs = np.random.RandomState(seed)
        u, p, n = recsys.sample_bpr_triplets_from_condensed(pl, ni, batch, rs)
        assert np.array_equal(u, z[f"s{c}_u"]) and np.array_equal(p, z[f"s{c}_pos"])
        assert np.array_equal(n, z[f"s{c}_neg"])
        st = rs.get_state(legacy=True)
        assert np.array_equal(st[1], z[f"s{c}_key"]) and st[2] == int(z[f"s{c}_statepos"])
        # the reference's own input form (a list of arrays) goes through the same native draws
        u2, p2, n2 = recsys.sample_bpr_triplets_from_condensed(rows, ni, batch, np.random.RandomState(seed))
        assert np.array_equal(u2, u) and np.array_equal(p2, p) and np.array_equal(n2, n)


def test_native_bpr_sampler_unsorted_lists_vs_oracle():
    recsys = _gdd()
    rng = np.random.default_rng(5)
    rows = [rng.permutation(50)[:rng.integers(0, 12)] for _ in range(40)]
    rows[3] = np.arange(50)[::-1]  # a full list, descending
    for seed in (0, 1, 2):
        a = recsys.sample_bpr_triplets_from_condensed(rows, 50, 700, np.random.RandomState(seed))
        b = R.bpr_triplets(rows, 50, 700, np.random.RandomState(seed))
        assert all(np.array_equal(x, y) for x, y in zip(a, b))


def test_recall_oracle_vs_reference_without_ties():
    import scipy.sparse as sp
    z = load("golden_refine.npz")
    ue, ie = z["r0_ue"], z["r0_ie"]
    Rtr = sp.coo_matrix((np.ones(z["r0_tr_u"].shape[0], np.float32), (z["r0_tr_u"], z["r0_tr_i"])),
                        shape=(ue.shape[0], ie.shape[0])).tocsr()
    r = R.recall(ue, ie, Rtr.indptr, Rtr.indices, z["r0_te_u"], z["r0_te_i"], 20, max_users=250)
    assert r == float(z["r0_recall"])
