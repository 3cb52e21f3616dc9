"""CPU restatement (test infrastructure only) of the recommender condensation of ClustGDD.

build_condensed_bipartite follows ClustGDD/distill_recsys.py:184-201: super-node pairs
(u2cu[u], i2ci[i]) of the interactions, pair counts summed (scipy coo -> sum_duplicates -> tocsr), i.e.
canonical CSR with rows and columns ascending and fp32 counts. Pinned by tests/golden/golden_recsys.npz
(G8, produced by the reference function itself, tools/make_golden.py).
"""
import numpy as np


def build_condensed_bipartite(train_u, train_i, u2cu, i2ci, num_cu: int, num_ci: int):
    """-> (rowptr int64 [num_cu+1], col int64 [nnz], val fp32 [nnz])."""
    cu = np.asarray(u2cu, np.int64)[np.asarray(train_u, np.int64)]
    ci = np.asarray(i2ci, np.int64)[np.asarray(train_i, np.int64)]
    key = cu * int(num_ci) + ci
    uniq, counts = np.unique(key, return_counts=True)
    rows, cols = uniq // int(num_ci), uniq % int(num_ci)
    rowptr = np.zeros(int(num_cu) + 1, np.int64)
    np.add.at(rowptr, rows + 1, 1)
    return np.cumsum(rowptr), cols, counts.astype(np.float32)
