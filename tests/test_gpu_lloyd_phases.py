"""The Lloyd loop's phase entry points (gdd_lloyd_estep / _mstep / _update) on one GPU.

* The convergence test's numpy pairwise sum of the squared centre shifts, evaluated by the workgroup
  (leaves in parallel, r04): with tol set to numpy's own float32 sum S, the loop stops (reason 2);
  with tol one ulp below S it does not — for k across the leaf-layout cases (fewer than 8 values, one
  leaf, leaf boundaries, many leaves).
* The M-step over a feature-column range equals the corresponding columns of the full fold, for the
  small-cluster (8 KiB chunk) and the regular fold buffers.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

from gdd import _lib  # noqa: E402


@pytest.mark.parametrize("k", [1, 5, 7, 8, 9, 100, 128, 129, 135, 604, 1000, 1773, 5000, 8192])
def test_update_convergence_sum_is_numpys(k):
    lib = _lib.device_lib()
    dim, n = 3, 16
    rng = np.random.default_rng(k)
    C_old = rng.standard_normal((k, dim)).astype(np.float32)
    C_new = (C_old + rng.standard_normal((k, dim)).astype(np.float32) * np.float32(1e-3)
             * rng.random((k, 1)).astype(np.float32) ** 4).astype(np.float32)
    wsum = np.ones(k, np.float32)  # averaging by 1/1 leaves C_new as it is
    dev = "cuda"
    shift = torch.empty(k, dtype=torch.float32, device=dev)
    labels = torch.zeros(n, dtype=torch.int32, device=dev)
    res = []
    for pick in ("at", "below"):
        Cn = torch.from_numpy(C_new.copy()).to(dev)
        Co = torch.from_numpy(C_old).to(dev)
        w = torch.from_numpy(wsum).to(dev)
        labels_old = torch.full((n,), -1, dtype=torch.int32, device=dev)  # changed: the tol test decides
        state = torch.zeros(lib.gdd_lloyd_state_bytes(), dtype=torch.uint8, device=dev)
        # first pass with tol = -1 (never stops) to read the shifts the device computes
        _lib.check(lib.gdd_lloyd_update(n, dim, k, None, 1, Cn.data_ptr(), w.data_ptr(), Co.data_ptr(),
                                        shift.data_ptr(), labels.data_ptr(), labels_old.data_ptr(), -1.0,
                                        state.data_ptr(), 0, _lib.stream_ptr()))
        sh = shift.cpu().numpy()
        S = float(np.sum(sh * sh, dtype=np.float32))  # numpy's pairwise float32 sum
        tol = S if pick == "at" else float(np.nextafter(np.float32(S), np.float32(0)))
        Cn = torch.from_numpy(C_new.copy()).to(dev)
        labels_old = torch.full((n,), -1, dtype=torch.int32, device=dev)
        state = torch.zeros(lib.gdd_lloyd_state_bytes(), dtype=torch.uint8, device=dev)
        _lib.check(lib.gdd_lloyd_update(n, dim, k, None, 1, Cn.data_ptr(), w.data_ptr(), Co.data_ptr(),
                                        shift.data_ptr(), labels.data_ptr(), labels_old.data_ptr(), tol,
                                        state.data_ptr(), 0, _lib.stream_ptr()))
        st = state[:20].view(torch.int32).cpu().numpy()
        res.append((int(st[0]), int(st[1])))
    assert res[0] == (2, 2), res  # stop_at = step 1 + 1, reason 2 (tol)
    assert res[1] == (0, 0), res


@pytest.mark.parametrize("n,dim,k", [(6040, 64, 604), (20000, 47, 196), (3000, 41, 40)])
def test_mstep_column_range_equals_full_fold(n, dim, k):
    """Each rank's column slice (gdd_lloyd_mstep over [f0, f1)) is exactly those columns of the full
    ordered fold and of the oracle's segment sums."""
    lib = _lib.device_lib()
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, dim)).astype(np.float32)
    lab = rng.integers(0, k, n).astype(np.int32)
    lab[: k] = np.arange(k)  # no empty cluster
    ref = np.empty((k, dim), np.float32)
    wref = np.empty(k, np.float32)
    O.lib().oracle_segment_sum_f32(n, dim, X, None, lab, k, ref, wref)
    Xd, ld = torch.from_numpy(X).cuda(), torch.from_numpy(lab).cuda()
    ws = _lib.workspace(lib.gdd_kmeans_lloyd_ws_bytes(n, dim, k), Xd.device)
    for f0, f1 in [(0, dim), (0, (dim + 1) // 2), ((dim + 1) // 2, dim), (dim - 3, dim)]:
        state = torch.zeros(lib.gdd_lloyd_state_bytes(), dtype=torch.uint8, device="cuda")
        out = torch.empty(k * (f1 - f0), dtype=torch.float32, device="cuda")
        wsum = torch.empty(k, dtype=torch.float32, device="cuda")
        _lib.check(lib.gdd_lloyd_mstep(n, dim, Xd.data_ptr(), ld.data_ptr(), k, f0, f1, out.data_ptr(),
                                       wsum.data_ptr(), state.data_ptr(), 0, ws.data_ptr(), ws.numel(),
                                       _lib.stream_ptr()))
        got = out.cpu().numpy().reshape(k, f1 - f0)
        assert np.array_equal(got.view(np.uint32), np.ascontiguousarray(ref[:, f0:f1]).view(np.uint32))
        assert np.array_equal(wsum.cpu().numpy(), wref)
