#!/usr/bin/env python3
"""Config 4 end to end (distill_recsys.py main at the MovieLens-1M shape) on the device: the drop-in
driver gdd.distill_recsys.run with the reference's default flags (reduction 0.1, KMeans on SVD-64
embeddings, 500 BPR refinement epochs of batch 4096, Recall@20 every 50 epochs), on a synthetic
Rankformer-format dataset: 6,040 users, 3,706 items, 1,000,209 unique interactions (80/10/10
split), power-law user activity and item popularity. SVD embeddings: scipy svds on the host (timed, as in the reference).

Prints the driver's own stdout and one JSON line with per-stage wall times.
usage: bench_recsys_e2e.py [epochs]
       bench_recsys_e2e.py alidisplay [epochs]   the real Rankformer/data/Ali-Display files (from the
           fixture tests/golden/golden_alidisplay.npz, with the reference's captured SVD embeddings),
           the reference's default flags; the JSON line carries both Recall@20 trajectories"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gdd import distill_recsys as D  # noqa: E402
from gdd import kmeans as K  # noqa: E402


def warm_kmeans(args, user_emb, item_emb, num_cu, num_ci, reps=3):
    """The clustering stage again in the same process (libraries loaded, workspaces cached): per call
    wall time and gdd.kmeans phases — against the driver's first-call kmeans_s."""
    out = {}
    for name, emb, k in (("users", user_emb, num_cu), ("items", item_emb, num_ci)):
        best = None
        for _ in range(reps):
            K.PHASE_TIMING = {}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            D.kmeans_cluster(emb, n_clusters=k, seed=args.seed, minibatch=args.kmeans_minibatch,
                             batch_size=args.kmeans_batch_size, device="cuda")
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            if best is None or ms < best["ms"]:
                best = {"ms": ms, "phases_ms": dict(K.PHASE_TIMING)}
        K.PHASE_TIMING = None
        out[name] = best
    return out


def write_dataset(root, nu=6040, ni=3706, E=1000209, seed=4):
    """Power-law user activity and item popularity (rank^-0.5 / rank^-0.8), de-duplicated and cut
    to E unique (user, item) pairs."""
    rng = np.random.default_rng(seed)
    wu = np.arange(1, nu + 1, dtype=np.float64) ** -0.5
    wi = np.arange(1, ni + 1, dtype=np.float64) ** -0.8
    u = rng.permutation(nu)[rng.choice(nu, int(E * 1.6), p=wu / wu.sum())]
    it = rng.permutation(ni)[rng.choice(ni, int(E * 1.6), p=wi / wi.sum())]
    key = np.unique(u.astype(np.int64) * ni + it)
    key = key[rng.permutation(key.shape[0])[:E]]
    pairs = np.stack([key // ni, key % ni], 1)
    n = pairs.shape[0]
    a, b = int(0.8 * n), int(0.9 * n)
    os.makedirs(os.path.join(root, "ml1m"))
    for name, part in (("train", pairs[:a]), ("valid", pairs[a:b]), ("test", pairs[b:])):
        np.savetxt(os.path.join(root, "ml1m", f"{name}.txt"), part, fmt="%d")
    return n


def main(epochs=500):
    with tempfile.TemporaryDirectory() as tmp:
        n = write_dataset(tmp)
        args = D.parse_args(["--data_dir", tmp, "--dataset", "ml1m", "--refine_epochs", str(epochs)])
        tm = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        D.run(args, out_root=os.path.join(tmp, "out"), timings=tm)
        torch.cuda.synchronize()
        tm["total_s"] = time.perf_counter() - t0
        ds = D.load_rankformer_dataset(tmp, "ml1m")
        R_train = D.build_interaction_matrix(ds.num_users, ds.num_items, ds.train_u, ds.train_i)
        ue, ie = D.compute_svd_embeddings(R_train, dim=args.svd_dim, seed=args.seed)
        tm["kmeans_warm"] = warm_kmeans(args, ue, ie, int(np.ceil(ds.num_users * args.reduction_rate)),
                                        int(np.ceil(ds.num_items * args.reduction_rate)))
    tm["refine_ms_per_epoch"] = tm["refine_s"] / max(1, epochs) * 1e3
    print(json.dumps({"workload": f"distill_recsys main, ML-1M shape: 6040 users x 3706 items, {n} unique "
                                  f"interactions, reduction 0.1, svd 64, KMeans, {epochs} BPR epochs b=4096",
                      **tm}), flush=True)


def alidisplay(epochs=500):
    """The drop-in driver on the reference's real dataset beside the reference's own trajectory."""
    import contextlib
    import io
    z = np.load(os.path.join(ROOT, "tests", "golden", "golden_alidisplay.npz"))
    ref = open(os.path.join(ROOT, "tests", "golden", "golden_alidisplay_full_stdout.txt")).read().splitlines()
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "Ali-Display"))
        for split in ("train", "valid", "test"):
            np.savetxt(os.path.join(tmp, "Ali-Display", f"{split}.txt"),
                       np.stack([z[f"{split}_u"], z[f"{split}_i"]], 1), fmt="%d")
        args = D.parse_args(["--data_dir", tmp, "--dataset", "Ali-Display", "--refine_epochs", str(epochs)])
        tm = {}
        buf = io.StringIO()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(buf):
            D.run(args, out_root=os.path.join(tmp, "out"), timings=tm,
                  embeddings=(z["user_emb"], z["item_emb"]))
        torch.cuda.synchronize()
        tm["total_s"] = time.perf_counter() - t0
        tm["kmeans_warm"] = warm_kmeans(args, z["user_emb"], z["item_emb"], 1773, 1004)
    out = buf.getvalue().splitlines()
    print("\n".join(out))

    def traj(lines):
        return [(l.split()[1], float(l.rsplit("=", 1)[1])) for l in lines if l.startswith("[refine] ep=")]
    tm["refine_ms_per_epoch"] = tm["refine_s"] / max(1, epochs) * 1e3
    print(json.dumps({"workload": f"distill_recsys main on the real Ali-Display data (17,730 users x 10,036 "
                                  f"items, 121,178 train interactions), default flags, {epochs} BPR epochs",
                      **tm, "recall_gpu": traj(out), "recall_reference_cpu": traj(ref),
                      "loss_gpu": [float(l.split("loss=")[1].split()[0]) for l in out if "loss=" in l],
                      "loss_reference_cpu": [float(l.split("loss=")[1].split()[0]) for l in ref if "loss=" in l]}),
          flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["alidisplay"]:
        alidisplay(*(int(a) for a in sys.argv[2:3]))
    else:
        main(*(int(a) for a in sys.argv[1:2]))
