"""ctypes binding of libgdd.so (the C ABI declared in include/gdd.h).

PyTorch provides device memory and the stream; every call passes raw device pointers and the
current HIP stream to the library. There is no CPU fallback: if the library or a gfx950 device is
missing, the first call raises.

torch is imported before the library is loaded on purpose: torch ships its own libamdhip64.so
(SONAME libamdhip64.so.7); loading libgdd.so afterwards makes the dynamic loader reuse that same
runtime instead of pulling a second copy from /opt/rocm.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# GDD_LIB_PATH selects a diagnostic build of the same library (e.g. lib/libgdd_stamps.so)
LIB_PATH = os.environ.get("GDD_LIB_PATH") or os.path.join(_HERE, "lib", "libgdd.so")

_c_i64 = ctypes.c_int64
_c_int = ctypes.c_int
_c_f32 = ctypes.c_float
_c_size = ctypes.c_size_t
_vp = ctypes.c_void_p

# name -> (restype, argtypes); kept in the order of include/gdd.h
SIGNATURES = {
    "gdd_last_error": (ctypes.c_char_p, []),
    "gdd_abi_version": (_c_int, []),
    "gdd_spin_limit": (_c_int, []),
    "gdd_device_ok": (_c_int, []),
    "gdd_normalize_ws_bytes": (_c_size, [_c_i64, _c_i64]),
    "gdd_normalize_csr": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, _vp,
                                   _c_size, _vp]),
    "gdd_propagate_ws_bytes": (_c_size, [_c_i64, _c_i64, _c_int]),
    "gdd_propagate": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _c_int, _vp, _c_int, _c_f32, _vp,
                               _vp, _vp, _vp, _c_size, _vp]),
    "gdd_propagate_relabeled_ws_bytes": (_c_size, [_c_i64, _c_i64, _c_int]),
    "gdd_propagate_relabeled": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_int, _vp, _c_int, _c_f32,
                                         _vp, _vp, _vp, _vp, _c_size, _vp]),
    "gdd_spmm": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _c_int, _c_f32, _vp, _vp, _vp, _c_f32,
                          _vp, _c_size, _vp]),
    "gdd_spmm_plan": (_c_int, [_c_i64, _c_i64, _vp, _c_int, _vp, _c_size, _vp]),
    "gdd_spmm_planned": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _c_int, _c_f32, _vp, _vp, _vp,
                                  _c_f32, _vp, _c_size, _vp]),
    "gdd_row_norms": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp]),
    "gdd_kmeans_assign_ws_bytes": (_c_size, [_c_i64]),
    "gdd_kmeans_assign": (_c_int, [_c_i64, _c_int, _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _vp,
                                   _c_size, _vp]),
    "gdd_kmeans_assign_bf16": (_c_int, [_c_i64, _c_int, _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _vp,
                                   _c_size, _vp]),
    "gdd_inertia": (_c_int, [_c_i64, _vp, _vp, _vp, _vp]),
    "gdd_inertia_ws_bytes": (_c_size, [_c_i64]),
    "gdd_inertia_ws": (_c_int, [_c_i64, _vp, _vp, _vp, _vp, _c_size, _vp]),
    "gdd_minibatch_update_ws_bytes": (_c_size, [_c_i64, _c_int]),
    "gdd_minibatch_update": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp,
                                      _vp, _c_size, _vp]),
    "gdd_minibatch_state_bytes": (_c_size, []),
    "gdd_minibatch_step_ws_bytes": (_c_size, [_c_i64, _c_int]),
    "gdd_minibatch_step": (_c_int, [_c_i64, _c_int, _vp, _vp, _c_int, _vp, _vp, _vp, _vp, _c_int,
                                    _c_i64, _c_int, _c_int, _vp, _vp, _c_size, _vp]),
    "gdd_minibatch_converge": (_c_int, [_c_i64, _c_int, _c_int, _c_i64, _c_int, _vp, _vp, _c_size,
                                        _vp]),
    "gdd_minibatch_kmeans_fit_ws_bytes": (_c_size, [_c_i64, _c_int, _c_int, _c_i64, _c_i64]),
    "gdd_minibatch_kmeans_fit": (_c_int, [_c_i64, _c_int, _vp, _c_int, _c_i64, _c_int, _c_int,
                                          _c_f32, _c_i64, _c_int, _c_int, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _vp, _vp, _c_size, _vp, _c_size, _vp]),
    "gdd_minibatch_kmeans_fit_host_ws_bytes": (_c_size, [_c_i64, _c_int, _c_i64, _c_i64]),
    "gdd_rng_randint": (_c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp]),
    "gdd_rng_random_sample": (_c_int, [_vp, _c_i64, _vp]),
    "gdd_rng_permutation": (_c_int, [_vp, _c_i64, _vp]),
    "gdd_rng_choice_unit_weights": (_c_int, [_vp, _c_i64, _vp]),
    "gdd_group_ws_bytes": (_c_size, [_c_i64, _c_int]),
    "gdd_group_by_label": (_c_int, [_c_i64, _vp, _c_int, _vp, _vp, _vp, _c_size, _vp]),
    "gdd_segment_sum_f32": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp]),
    "gdd_segment_sum_f32_part": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _vp, _c_int, _c_int, _c_int,
                                          _vp, _vp, _vp]),
    "gdd_average_centers": (_c_int, [_c_int, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "gdd_point_center_sqdist": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "gdd_relocate_distances": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "gdd_lloyd_state_bytes": (_c_size, []),
    "gdd_kmeans_lloyd_ws_bytes": (_c_size, [_c_i64, _c_int, _c_int]),
    "gdd_kmeans_lloyd_host_ws_bytes": (_c_size, []),
    "gdd_kmeans_lloyd_run": (_c_int, [_c_i64, _c_int, _vp, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _c_int,
                                      _c_int, _c_int, ctypes.c_double, _vp, _vp, _vp, _vp, _c_size,
                                      _vp, _c_size, _vp]),
    "gdd_lloyd_estep": (_c_int, [_c_i64, _c_i64, _c_i64, _c_int, _vp, _c_int, _vp, _vp, _c_int, _vp,
                                 _vp, _c_int, _vp, _c_size, _vp]),
    "gdd_lloyd_mstep": (_c_int, [_c_i64, _c_int, _vp, _vp, _c_int, _c_int, _c_int, _vp, _vp, _vp,
                                 _c_int, _vp, _c_size, _vp]),
    "gdd_lloyd_update": (_c_int, [_c_i64, _c_int, _c_int, _vp, _c_int, _vp, _vp, _vp, _vp, _vp, _vp,
                                  ctypes.c_double, _vp, _c_int, _vp]),
    "gdd_skl_sqdist": (_c_int, [_c_int, _vp, _c_i64, _c_int, _vp, _vp, _vp]),
    "gdd_kmeans_plusplus_ws_bytes": (_c_size, [_c_i64, _c_int, _c_int]),
    "gdd_kmeans_plusplus_ws_bytes_k": (_c_size, [_c_i64, _c_int, _c_int, _c_int]),
    "gdd_kmeans_plusplus": (_c_int, [_c_i64, _c_int, _vp, _vp, _c_int, _c_int, _c_i64, _vp, _vp,
                                     _vp, _vp, _c_size, _vp]),
    "gdd_standard_scaler": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "gdd_center_columns": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "gdd_center_columns_ws_bytes": (_c_size, [_c_i64, _c_int]),
    "gdd_center_columns_ws": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _vp, _vp, _c_size, _vp]),
    "gdd_standard_scaler_transform": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _vp, _vp]),
    "gdd_cluster_mean": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _c_int, _c_int, _vp, _vp, _vp]),
    "gdd_cluster_mean_part": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp, _c_int, _c_int, _c_int, _c_int,
                                       _vp, _vp, _vp]),
    "gdd_argmax_rows": (_c_int, [_c_int, _c_int, _vp, _vp, _vp]),
    "gdd_coo_rows": (_c_int, [_c_i64, _vp, _vp, _vp]),
    "gdd_er_ws_bytes": (_c_size, [_c_i64, _c_int]),
    "gdd_attaw_er": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_int, _vp, _vp, _vp, _vp,
                              _c_size, _vp]),
    "gdd_vanilla_er": (_c_int, [_c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _c_size, _vp]),
    "gdd_softmax_rows": (_c_int, [_c_i64, _c_int, _vp, _vp, _vp]),
    "gdd_topk_ws_bytes": (_c_size, [_c_i64, _c_int]),
    "gdd_class_topk": (_c_int, [_c_i64, _vp, _vp, _vp, _c_int, _vp, _c_i64, _vp, _vp, _c_size,
                                _vp]),
    "gdd_compress_ws_bytes": (_c_size, [_c_int]),
    "gdd_graph_compress": (_c_int, [_c_i64, _vp, _c_int, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _c_size, _vp]),
    "gdd_stream_copy": (_c_int, [_vp, _vp, _c_size, _vp]),
    "gdd_csr_transpose_ws_bytes": (_c_size, [_c_i64, _c_i64, _c_i64]),
    "gdd_csr_transpose": (_c_int, [_c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _c_size, _vp]),
    "gdd_bipartite_condense_ws_bytes": (_c_size, [_c_i64, _c_int]),
    "gdd_bipartite_condense": (_c_int, [_c_i64, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_int, _c_int, _vp,
                                        _vp, _vp, _vp, _vp, _vp, _c_size, _vp]),
    "gdd_edge_dots": (_c_int, [_c_i64, _c_int, _vp, _vp, _c_i64, _vp, _vp, _c_i64, _vp, _vp, _vp]),
    "gdd_bpr_sample": (_c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp]),
    "gdd_recall_at_k": (_c_int, [_c_int, _c_i64, _c_int, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gdd_subgraph_ws_bytes": (_c_size, [_c_i64, _c_i64]),
    "gdd_subgraph_count": (_c_int, [_c_i64, _vp, _vp, _c_i64, _vp, _vp, _vp, _c_size, _vp]),
    "gdd_subgraph_fill": (_c_int, [_c_i64, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp, _vp, _vp, _vp,
                                   _c_size, _vp]),
    "gdd_select_csr_ws_bytes": (_c_size, [_c_i64]),
    "gdd_select_csr": (_c_int, [_c_i64, _vp, _vp, _vp, _c_i64, _vp, _vp, _vp, _vp, _vp, _c_size,
                                _vp]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load libgdd.so and attach signatures (no device work)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libgdd.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; "
            "g.build()'` (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


_device_checked = False


def device_lib() -> ctypes.CDLL:
    """The library, after checking that the current device is a gfx950 GPU."""
    global _device_checked
    lib = load()
    if not _device_checked:
        if not torch.cuda.is_available():
            raise RuntimeError("gdd: no HIP device visible; the MI355X path has no CPU fallback")
        torch.cuda.current_device()
        if lib.gdd_device_ok() != 1:
            name = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
            raise RuntimeError(f"gdd: device arch {name!r} is not gfx950")
        _device_checked = True
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().gdd_last_error().decode(errors="replace")
        raise RuntimeError(f"libgdd error {rc:#x}: {msg}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def pinned_workspace(nbytes: int) -> torch.Tensor:
    """Page-locked host staging from PyTorch's pinned caching allocator (no per-call hipHostMalloc)."""
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, pin_memory=True)


class MTState(ctypes.Structure):
    """gdd_mt_state: numpy's legacy RandomState state, passed to the native loops by pointer."""

    _fields_ = [("key", ctypes.c_uint32 * 624), ("pos", ctypes.c_int32),
                ("has_gauss", ctypes.c_int32), ("gauss", ctypes.c_double)]

    @classmethod
    def from_random_state(cls, rs):
        name, key, pos, has_gauss, gauss = rs.get_state(legacy=True)
        if name != "MT19937":
            raise ValueError(f"unsupported bit generator {name}")
        st = cls()
        key32 = key.astype("uint32")  # keep the array alive across the copy
        ctypes.memmove(st.key, key32.ctypes.data, 624 * 4)
        st.pos, st.has_gauss, st.gauss = int(pos), int(has_gauss), float(gauss)
        return st

    def to_random_state(self, rs):
        import numpy as np
        key = np.ctypeslib.as_array(self.key).copy()
        rs.set_state(("MT19937", key, int(self.pos), int(self.has_gauss), float(self.gauss)))


ARGSORT_CB = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_float), ctypes.c_int64,
                              ctypes.POINTER(ctypes.c_int64))


def _np_argsort(w_ptr, k, out_ptr):
    import numpy as np
    w = np.ctypeslib.as_array(w_ptr, shape=(k,)).copy()
    np.ctypeslib.as_array(out_ptr, shape=(k,))[:] = np.argsort(w)


# np.argsort(weight_sums) for the native MiniBatchKMeans loop (kept alive for the process)
argsort_callback = ARGSORT_CB(_np_argsort)
