#!/usr/bin/env python3
"""k-means++ seeding alone: device time per fit (HIP events) at the shapes the fits use, checked
against the oracle (indices and centres bit-exact)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-distillation-for-recommendation_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gdd import _lib, synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(n, dim, k, reps, check=True):
    lib = _lib.device_lib()
    s = _lib.stream_ptr()
    X = synth.blobs(n, dim, max(k // 4, 2), seed=n + dim)
    T = 2 + int(np.log(k))
    rs = np.random.RandomState(15)
    w = np.ones(n, np.float32)
    first = int(rs.choice(n, p=w / w.sum()))
    U = rs.uniform(size=(k - 1) * T)
    Xd = torch.from_numpy(X).cuda()
    Ud = torch.from_numpy(U).cuda()
    C = torch.empty(k, dim, dtype=torch.float32, device="cuda")
    idx = torch.empty(k, dtype=torch.int64, device="cuda")
    ws = _lib.workspace(lib.gdd_kmeans_plusplus_ws_bytes(n, dim, T), "cuda")

    def call():
        _lib.check(lib.gdd_kmeans_plusplus(n, dim, Xd.data_ptr(), None, k, T, first, Ud.data_ptr(),
                                           C.data_ptr(), idx.data_ptr(), ws.data_ptr(), ws.numel(), s))
    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    ok = ""
    if check:
        Cr, ir = O.kmeans_plusplus(X, k, np.random.RandomState(15))
        ok = "parity ok" if (np.array_equal(ir, idx.cpu().numpy()) and
                             np.array_equal(Cr, C.cpu().numpy())) else "PARITY MISMATCH"
    print(f"n={n:7d} dim={dim:4d} k={k:5d} T={T:2d}: {ms:8.3f} ms/fit  {ms * 1e3 / max(k - 1, 1):7.2f} us/round  {ok}",
          flush=True)


def ab(n=3000, dim=40, k=454):
    """Same-process A/B of the round forms (devices differ by up to ~10% in clock) through
    GDD_FORCE, and of the cumulative-potential rounding check (GDD_KPP_EXACT: 0 off, 1 default, 2
    replay every draw)."""
    for var, val in (("", ""), ("GDD_FORCE", "kpp_pair_serial"), ("GDD_FORCE", "kpp_single_round"),
                     ("GDD_FORCE", "kpp_no_table"), ("", ""), ("GDD_FORCE", "kpp_pair_serial"),
                     ("GDD_KPP_EXACT", "0"), ("", ""), ("GDD_KPP_EXACT", "2")):
        if var:
            os.environ[var] = val
        print(f"variant {var + '=' + val if var else 'default'}:", end=" ", flush=True)
        run(n, dim, k, 5, check=False)
        if var:
            del os.environ[var]


def ab_big():
    """One 1024-thread workgroup per trial (k_kpp1_big, default for 4096 < n <= 16384 table plans;
    two rounds per launch, k_kpp1_big2, up to n = 8192 with T <= 8) against one round per launch
    (GDD_FORCE=kpp_single_round) and the per-(block, trial) table rounds (kpp_no_big1), same process;
    the ML-1M users' shape parity-checked first."""
    run(6040, 64, 604, 1)
    for (n, dim, k) in [(6040, 64, 604), (8000, 64, 400), (9001, 24, 200), (17730, 64, 1773)]:
        for var in ("", "kpp_single_round", "kpp_no_big1", "", "kpp_single_round"):
            if var:
                os.environ["GDD_FORCE"] = var
            print(f"variant {var or 'default'}:", end=" ", flush=True)
            run(n, dim, k, 3, check=False)
            if var:
                del os.environ["GDD_FORCE"]


if __name__ == "__main__":
    if sys.argv[1:2] == ["arxiv"]:  # timing only: the bench's init shape, ML-1M users, Ali-Display users
        for (n, dim, k, reps) in [(3000, 40, 454, 5), (6040, 64, 604, 3), (17730, 64, 1773, 1)]:
            run(n, dim, k, reps, check=False)
        sys.exit(0)
    if sys.argv[1:2] == ["shape"]:  # timing only: micro_kpp.py shape n dim k [reps]
        n_, d_, k_ = (int(v) for v in sys.argv[2:5])
        run(n_, d_, k_, int(sys.argv[5]) if len(sys.argv) > 5 else 5, check=False)
        sys.exit(0)
    if sys.argv[1:2] == ["one"]:  # the MiniBatchKMeans init shape alone, parity checked
        run(3000, 40, 454, 5)
        sys.exit(0)
    if sys.argv[1:2] == ["big"]:
        ab_big()
        sys.exit(0)
    ab()
    for (n, dim, k) in [(3000, 40, 454), (2708, 7, 70), (3706, 64, 371), (6040, 64, 604), (3000, 41, 769),
                        (17730, 64, 1773)]:
        run(n, dim, k, 3, check=n * k < 3e7)
