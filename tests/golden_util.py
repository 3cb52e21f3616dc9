"""Loading helpers for the golden fixtures (tests/golden/, produced by tools/make_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Propagation parity against the reference's torch-CPU SpMM: its summation order is not the
# canonical one (nor cuSPARSE's), so fp32 results agree to rounding, not bit for bit.
PROP_RTOL, PROP_ATOL = 1e-5, 1e-6
# Cluster means: the reference reduces with torch.mean (fp32 tree); ours is fp64 then rounded.
MEAN_RTOL, MEAN_ATOL = 1e-5, 1e-6


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def graph_names():
    return ["binary", "selfloop0", "weighted", "isolated"]


def rng_from_fixture(z):
    """The numpy global-RNG state captured right before the reference's sklearn call."""
    rs = np.random.RandomState()
    rs.set_state(("MT19937", z["rng_key"], int(z["rng_pos"]), int(z["rng_has_gauss"]),
                  float(z["rng_cached_gauss"])))
    return rs


def csr_to_sorted_coo(rowptr, col, val):
    rows = np.repeat(np.arange(len(rowptr) - 1, dtype=np.int32), np.diff(rowptr))
    return rows, np.asarray(col, np.int32), np.asarray(val, np.float32)


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
