"""Drop-in for ``ClustGDD/distill_recsys.py`` (the recommender distillation driver, BASELINE config 4)
on libgdd: the same command-line flags, stdout lines, training loop and artefacts, with every
device step on the MI355X path.

    python -m gdd.distill_recsys --data_dir Rankformer/data --dataset Ali-Display

Stage by stage (reference line ranges):

1. data (:45-117): the Rankformer text files; the interaction matrix is a host scipy CSR;
2. embeddings (:124-155): ``scipy.sparse.linalg.svds`` on the host, as the reference does (its ARPACK
   start vector is the one thing here that is not seeded by ``--seed``; pass ``embeddings=`` to
   :func:`run` to use fixed ones);
3. clustering (:158-181, :560-583): :func:`gdd.pipeline.kmeans_cluster` (device StandardScaler and
   KMeans / MiniBatchKMeans, bit-exact with scikit-learn);
4. condensation (:184-201): :func:`gdd.recsys.build_condensed_bipartite` (device, bit-exact);
5. teacher KD (:592-638): the super-node means on the device (:func:`gdd.pipeline.teacher_means`);
6. refinement (:640-733): :class:`gdd.recsys.LightGCNCondensed` (SpMM message passing),
   :func:`gdd.recsys.sample_bpr_triplets_from_condensed` (native, the reference's draws),
   :func:`gdd.recsys.manual_adam_step`, :class:`gdd.recsys.RecallEvaluator` (device);
7. artefacts (:735-764): :func:`gdd.recsys.save_distilled`.

The reference falls back to the CPU when no GPU is visible; this driver has no CPU path.
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time
from dataclasses import dataclass
from typing import Optional

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn.functional as F

from . import recsys as R
from .pipeline import kmeans_cluster_pair, teacher_means


@dataclass
class RecDataset:
    """distill_recsys.RecDataset (:45-60)."""

    num_users: int
    num_items: int
    train_u: np.ndarray
    train_i: np.ndarray
    valid_u: np.ndarray
    valid_i: np.ndarray
    test_u: np.ndarray
    test_i: np.ndarray

    @property
    def num_edges_train(self) -> int:
        return int(self.train_u.shape[0])


def _read_pairs(path: str):
    a = np.loadtxt(path, dtype=np.int64).reshape(-1, 2) if os.path.getsize(path) else np.zeros((0, 2), np.int64)
    return a[:, 0].copy(), a[:, 1].copy()


def load_rankformer_dataset(data_dir: str, dataset: str) -> RecDataset:
    """``<data_dir>/<dataset>/{train,valid,test}.txt`` of "user item" lines (:63-107)."""
    root = os.path.join(data_dir, dataset)
    parts = {}
    for split in ("train", "valid", "test"):
        p = os.path.join(root, f"{split}.txt")
        if not os.path.exists(p):
            raise FileNotFoundError(f"Missing file: {p}")
        parts[split] = _read_pairs(p)
    nu = int(max(parts[s][0].max(initial=0) for s in parts) + 1)
    ni = int(max(parts[s][1].max(initial=0) for s in parts) + 1)
    print(f"[data] {dataset}: {nu} users, {ni} items")
    print(f"[data] edges train/valid/test: "
          f"{parts['train'][0].shape[0]}/{parts['valid'][0].shape[0]}/{parts['test'][0].shape[0]}")
    return RecDataset(nu, ni, *parts["train"], *parts["valid"], *parts["test"])


def build_interaction_matrix(num_users: int, num_items: int, u, i, values=None) -> sp.csr_matrix:
    """R (users x items) as scipy CSR (:110-117)."""
    v = np.ones(len(u), np.float32) if values is None else np.asarray(values, np.float32)
    return sp.coo_matrix((v, (u, i)), shape=(num_users, num_items)).tocsr()


def compute_svd_embeddings(R_: sp.csr_matrix, dim: int, seed: int = 42):
    """Truncated SVD embeddings scaled by sqrt(S) (:124-155), on the host like the reference."""
    from scipy.sparse.linalg import svds
    k = min(dim, min(R_.shape) - 1)
    if k <= 0:
        raise ValueError(f"Cannot compute SVD with shape={R_.shape} and dim={dim}")
    U, S, VT = svds(R_.astype(np.float64), k=k)
    order = np.argsort(S)[::-1]
    S, U, VT = S[order], U[:, order], VT[order, :]
    root = np.sqrt(np.maximum(S, 1e-12)).reshape(1, -1)
    return (U * root).astype(np.float32), (VT.T * root).astype(np.float32)


def parse_args(argv=None):
    """The reference's flags (:505-546), same names and defaults."""
    p = argparse.ArgumentParser()
    p.add_argument("--data_dir", type=str, default=os.path.join("Rankformer", "data"))
    p.add_argument("--dataset", type=str, default="Ali-Display")
    p.add_argument("--reduction_rate", type=float, default=0.1, help="keep rate for users/items (per-side).")
    p.add_argument("--svd_dim", type=int, default=64)
    p.add_argument("--kmeans_minibatch", action="store_true")
    p.add_argument("--kmeans_batch_size", type=int, default=2048)
    p.add_argument("--embed_dim", type=int, default=64)
    p.add_argument("--lgn_layers", type=int, default=2)
    p.add_argument("--refine_epochs", type=int, default=500)
    p.add_argument("--batch_size", type=int, default=4096)
    p.add_argument("--lr", type=float, default=1e-2)
    p.add_argument("--reg_lambda", type=float, default=1e-4)
    p.add_argument("--log_every", type=int, default=50)
    p.add_argument("--teacher_path", type=str, default=None,
                   help="Path to teacher Rankformer embeddings (.pt with user_emb/item_emb).")
    p.add_argument("--kd_lambda", type=float, default=0.01,
                   help="Weight for KD loss (MSE between student and aggregated teacher embeddings).")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--device", type=str, default="cuda")
    p.add_argument("--eval_topk", type=int, default=20)
    p.add_argument("--eval_max_users", type=int, default=5000)
    return p.parse_args(argv)


def run(args, out_root: str = "ClustGDD", embeddings=None, timings: Optional[dict] = None, group=None):
    """The reference's main() body (:548-764). ``embeddings``: optional fixed (user, item) SVD
    embeddings; ``timings``: filled with per-stage wall seconds; ``group``: a process group over the
    node's GPUs for the clustering pair (rank 0 users, rank 1 items). Returns the trained model."""
    tm = timings if timings is not None else {}
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    if not torch.cuda.is_available():
        raise RuntimeError("gdd.distill_recsys: no HIP device visible (the MI355X path has no CPU fallback)")
    device = torch.device(args.device if args.device.startswith("cuda") else "cuda")
    print(f"[env] device={device}")

    ds = load_rankformer_dataset(args.data_dir, args.dataset)
    R_train = build_interaction_matrix(ds.num_users, ds.num_items, ds.train_u, ds.train_i)

    print("[cluster] computing SVD embeddings...")
    t0 = time.perf_counter()
    if embeddings is None:
        user_emb_np, item_emb_np = compute_svd_embeddings(R_train, dim=args.svd_dim, seed=args.seed)
    else:
        user_emb_np, item_emb_np = embeddings
    tm["svd_s"] = time.perf_counter() - t0

    num_cu = max(1, int(math.ceil(ds.num_users * args.reduction_rate)))
    num_ci = max(1, int(math.ceil(ds.num_items * args.reduction_rate)))
    print(f"[cluster] target super nodes: users={num_cu}, items={num_ci}")
    t0 = time.perf_counter()
    print("[cluster] kmeans users...")
    print("[cluster] kmeans items...")
    # the two fits are independent (each random_state=seed): with a group, users on rank 0 and items
    # on rank 1, the results broadcast (gdd.pipeline.kmeans_cluster_pair; north star config 4)
    (u2cu, _), (i2ci, _) = kmeans_cluster_pair(user_emb_np, item_emb_np, num_cu, num_ci, seed=args.seed,
                                              minibatch=args.kmeans_minibatch,
                                              batch_size=args.kmeans_batch_size, device=device,
                                              group=group)
    u2cu, i2ci = np.asarray(u2cu, np.int64), np.asarray(i2ci, np.int64)
    torch.cuda.synchronize()
    tm["kmeans_s"] = time.perf_counter() - t0

    print("[compress] building condensed bipartite graph...")
    t0 = time.perf_counter()
    C = R.build_condensed_bipartite(ds.train_u, ds.train_i, u2cu, i2ci, num_cu, num_ci, device=device)
    nnz = C.nnz
    print(f"[compress] condensed edges: nnz={nnz}, density={float(nnz / max(1, num_cu * num_ci)):.6f}")
    torch.cuda.synchronize()
    tm["condense_s"] = time.perf_counter() - t0

    t_user = t_item = None
    if args.teacher_path is not None:
        if not os.path.exists(args.teacher_path):
            raise FileNotFoundError(f"Teacher file not found: {args.teacher_path}")
        print(f"[teacher] loading teacher embeddings from: {args.teacher_path}")
        data = torch.load(args.teacher_path, map_location="cpu", weights_only=True)
        if "user_emb" not in data or "item_emb" not in data:
            raise KeyError("teacher file must contain 'user_emb' and 'item_emb' tensors")
        tu, ti = data["user_emb"].to(device), data["item_emb"].to(device)
        if tu.shape[0] != ds.num_users or ti.shape[0] != ds.num_items:
            raise ValueError(f"Teacher emb size mismatch: user_emb {tu.shape[0]} vs {ds.num_users}, "
                             f"item_emb {ti.shape[0]} vs {ds.num_items}")
        if int(tu.shape[1]) != args.embed_dim:
            raise ValueError(f"Teacher embedding dim ({int(tu.shape[1])}) != student embed_dim "
                             f"({args.embed_dim}). Please re-train/save teacher with dim={args.embed_dim} "
                             "or add a projection layer.")
        print("[teacher] aggregating teacher embeddings to super-nodes (mean pooling)...")
        t_user = teacher_means(tu, u2cu, num_cu)
        t_item = teacher_means(ti, i2ci, num_ci)
        print("[teacher] KD will be applied during refinement.")

    pos_items_by_user = R._csr_row_to_set_list(C)
    edge_index, edge_weight_init = R.condensed_csr_to_edge_index(C, device=device)
    model = R.LightGCNCondensed(num_cu=num_cu, num_ci=num_ci, dim=args.embed_dim, num_layers=args.lgn_layers,
                                edge_index=edge_index, edge_weight_init=edge_weight_init,
                                device=device).to(device)
    params = [p for p in model.parameters() if p.requires_grad]
    adam_state: dict = {}
    rng = np.random.RandomState(args.seed)
    u2cu_t = torch.from_numpy(u2cu).to(device)
    i2ci_t = torch.from_numpy(i2ci).to(device)
    evaluator = R.RecallEvaluator(R_train, ds.test_u, ds.test_i, args.eval_topk, device, args.eval_max_users)

    def evaluate():
        cu_z, ci_z = model.propagate()
        return evaluator(cu_z[u2cu_t], ci_z[i2ci_t])

    with torch.no_grad():
        r0 = evaluate()
    print(f"[eval] Recall@{args.eval_topk} before refinement: {r0:.6f}")

    print("[refine] optimizing condensed graph with BPR loss...")
    model.train()
    t0 = time.perf_counter()
    for ep in range(1, args.refine_epochs + 1):
        u_np, pos_np, neg_np = R.sample_bpr_triplets_from_condensed(pos_items_by_user, num_ci,
                                                                    args.batch_size, rng)
        u = torch.from_numpy(u_np).to(device)
        pos_i = torch.from_numpy(pos_np).to(device)
        neg_i = torch.from_numpy(neg_np).to(device)
        loss = model.bpr_loss(u, pos_i, neg_i, reg_lambda=args.reg_lambda)
        if t_user is not None:
            su, si = model.propagate()
            loss = loss + args.kd_lambda * (F.mse_loss(su, t_user) + F.mse_loss(si, t_item))
        loss.backward()
        R.manual_adam_step(params, adam_state, lr=args.lr, step=ep)
        model.zero_grad(set_to_none=True)
        if ep % args.log_every == 0 or ep == 1 or ep == args.refine_epochs:
            model.eval()
            with torch.no_grad():
                r = evaluate()
            model.train()
            model.graph().check()  # at a point that synchronises anyway: no edge row id out of range
            print(f"[refine] ep={ep:04d} loss={loss.item():.6f} Recall@{args.eval_topk}={r:.6f}")
    torch.cuda.synchronize()
    tm["refine_s"] = time.perf_counter() - t0

    out_dir = os.path.join(out_root, "distilled_recsys", args.dataset)
    R.save_distilled(out_dir, model, u2cu, i2ci, num_cu, num_ci)
    print(f"[save] distilled artifacts saved to: {out_dir}")
    return model


def main(argv=None):
    run(parse_args(argv))


if __name__ == "__main__":
    main(sys.argv[1:])
