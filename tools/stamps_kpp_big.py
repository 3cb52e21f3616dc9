#!/usr/bin/env python3
"""In-kernel phase stamps of the multi-block k-means++ round (k_kpp_round, n > 4096) at the
products k-means shape (diagnostic build: make -C graph-distillation-for-recommendation_amd/csrc STAMPS=1).
Slots (block 0, trial 0, the last round): 20 start, 21 potentials folded, 22 block search done,
23 candidate counted, 24 distances written, 25 block terms written."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GDD_LIB_PATH"] = os.path.join(ROOT, "graph-distillation-for-recommendation_amd", "gdd", "lib",
                                          "libgdd_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gdd import _lib, synth  # noqa: E402
from gdd.kmeans import _Ops  # noqa: E402


def main(n=2449029, dim=47, k=24):
    lib = _lib.device_lib()
    X = torch.from_numpy(synth.blobs(n, dim, 196, seed=2)).cuda()
    ops = _Ops("cuda", n, k, dim)
    for _ in range(2):
        ops.kmeans_plusplus(X, k, np.random.RandomState(0))
        torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 256)()
    fn = lib.gdd_dbg_stamps_kpp
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
    assert fn(ctypes.addressof(buf)) == 0
    st = np.array(buf[:], dtype=np.int64)
    t0 = st[20]
    print("k_kpp_round phases (us): " + ", ".join(f"{q}: {(st[q] - t0) / 100:.2f}" for q in range(20, 26)))


if __name__ == "__main__":
    if len(sys.argv) == 4:  # n dim k, e.g. the Ali-Display users' per-block table rounds: 17730 64 1773
        main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]))
    else:
        main()
