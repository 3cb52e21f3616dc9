#!/usr/bin/env python3
"""In-kernel phase stamps (fused step: 60 start, 61 trip 1, 62 members sorted, 63 member rows in LDS,
64 chains done, 65 point tile ready, 66 keys out; 70-74 the same for an update alone) of the MiniBatchKMeans step and k-means++ kernels (diagnostic build).

Build: make -C graph-distillation-for-recommendation_amd/csrc STAMPS=1
Run:   python tools/stamps.py [kpp-big | kpp-dists]   (uses lib/libgdd_stamps.so; s_memrealtime, 10 ns ticks)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GDD_LIB_PATH"] = os.path.join(ROOT, "graph-distillation-for-recommendation_amd", "gdd", "lib",
                                          "libgdd_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import gdd  # noqa: E402
from gdd import _lib, synth  # noqa: E402


def read(lib, name):
    buf = (ctypes.c_ulonglong * 256)()
    fn = getattr(lib, "gdd_dbg_stamps_" + name)
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p]
    assert fn(ctypes.addressof(buf)) == 0
    return np.array(buf[:], dtype=np.int64)


def show(title, st, slots, base):
    t0 = st[base]
    parts = [f"{s}:{(st[s] - t0) * 10 / 1000:.2f}" for s in slots if st[s] >= t0 and st[s] - t0 < 10 ** 7]
    print(f"{title:22s} (us from slot {base}) " + " ".join(parts), flush=True)


def kpp_big():
    """k_kpp1_big's phases in round k-2 (trial 0) and the start of round k-1 (us)."""
    lib = _lib.device_lib()
    from gdd.kmeans import _Ops
    for (n, dim, k) in [(6040, 64, 604), (17730, 64, 1773)]:
        X = torch.from_numpy(synth.blobs(n, dim, k // 4, seed=n + dim)).cuda()
        for rep in range(2):
            _Ops("cuda", n, k, dim).kmeans_plusplus(X, k, np.random.RandomState(15))
            torch.cuda.synchronize()
            p = read(lib, "kpp")
            t0 = p[90]
            lab = {90: "start", 91: "winner + candidate", 92: "rows in LDS", 93: "prefix + chains",
                   96: "potential", 97: "draws", 94: "candidates out", 95: "next start"}
            print(f"n={n} k={k} rep {rep} (us): " + ", ".join(
                f"{lab[q]} {(p[q] - t0) / 100:.2f}" for q in [90, 91, 92, 93, 96, 97, 94, 95]), flush=True)


def kpp_dists():
    """k_kpp_dists' phases at the products shape (round 5; block 0 and the last block, us from block 0's
    start): candidates in LDS, the fp64 chains over the LDS-DMA ring, distances written, block totals,
    the sgemv_t block term."""
    lib = _lib.device_lib()
    from gdd.kmeans import _Ops
    n, dim, k = 2449029, 47, 196
    X = torch.randn(n, dim, device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    lab = ["start", "cands", "chains", "dists", "totals", "sgemv"]
    for rep in range(3):
        _Ops("cuda", n, k, dim).kmeans_plusplus(X, k, np.random.RandomState(15))
        torch.cuda.synchronize()
        p = read(lib, "kpp")
        t0 = p[30]
        for base, who in ((30, "block 0"), (40, "last block")):
            print(f"rep {rep} {who} (us): " + ", ".join(f"{lab[q]} {(p[base + q] - t0) / 100:.2f}"
                                                      for q in range(6)), flush=True)
        print(f"rep {rep} last wave of any block ends {(p[46] - t0) / 100:.2f} us after block 0's start", flush=True)


def main():
    if sys.argv[1:2] == ["kpp-big"]:
        return kpp_big()
    if sys.argv[1:2] == ["kpp-dists"]:
        return kpp_dists()
    lib = _lib.device_lib()
    cfg = synth.CONFIGS["arxiv"]
    X = torch.from_numpy(synth.blobs(cfg.n, cfg.n_classes, cfg.k, seed=1)).cuda()
    for rep in range(2):
        torch.cuda.synchronize()
        # "nostop": no early stop, so the last step launches are real steps (their stamps complete)
        extra = dict(max_no_improvement=None, max_iter=1) if sys.argv[1:2] == ["nostop"] else {}
        km = gdd.MiniBatchKMeans(n_clusters=cfg.k, random_state=cfg.seed, batch_size=cfg.batch,
                                 **extra).fit(X)
        torch.cuda.synchronize()
        a = read(lib, "kmeans")
        p = read(lib, "kpp")
        print(f"rep {rep}: steps={km.n_steps_}")
        show("fused step block0", a, list(range(60, 67)), 60)
        show("update alone block0", a, list(range(70, 75)), 70)
        show("assign_small", a, [0, 2, 3, 4, 5, 6, 13, 14, 15, 16, 82, 80, 83, 81], 0)
        show("update block0", a, list(range(20, 26)), 20)
        show("update tail", a, list(range(30, 33)), 30)
        show("mb_reassign", a, list(range(40, 47)), 40)
        show(f"reassign m={a[57]}", a, list(range(50, 57)), 50)
        show("reassign r05 forms", a, [48, 49, 64, 65, 59, 58], 48)  # shuffle start, end, mid stored, drawn, copies, draw stored
        print(f"block shuffle: {a[62]} Jacobi iterations, final pos {a[63]}")
        t0 = p[60]
        lab = {60: "start", 61: "winners resolved", 62: "level-1 fold done", 63: "level-2 row in LDS",
               75: "wave-1 prefix done", 76: "wave-0 chains done", 77: "wave-1 speculative searches done",
               70: "fold barrier", 74: "search+table", 65: "next start"}
        print("kpp pair launch (rounds k-3, k-2) (us): " + ", ".join(
            f"{lab[q]} {(p[q] - t0) / 100:.2f}" for q in [60, 61, 62, 63, 75, 76, 77, 70, 74, 65]
            if p[q] >= t0 and p[q] - t0 < 10 ** 6))


if __name__ == "__main__":
    main()
