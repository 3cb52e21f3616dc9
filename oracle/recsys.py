"""CPU restatement (test infrastructure only) of the recommender condensation of ClustGDD.

build_condensed_bipartite follows ClustGDD/distill_recsys.py:184-201: super-node pairs
(u2cu[u], i2ci[i]) of the interactions, pair counts summed (scipy coo -> sum_duplicates -> tocsr), i.e.
canonical CSR with rows and columns ascending and fp32 counts. Pinned by tests/golden/golden_recsys.npz
(G8, produced by the reference function itself, tools/make_golden.py).

The refinement loop's helpers (G11, golden_refine.npz, also from the reference's own functions):
bpr_triplets restates sample_bpr_triplets_from_condensed (distill_recsys.py:217-272) draw for draw on a
numpy RandomState; recall restates recall_at_k (:446-497) with one tie rule fixed (equal scores rank in
ascending item order; torch.topk leaves it unspecified).
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


def bpr_triplets(rows, num_items: int, batch: int, rs: np.random.RandomState):
    """-> (u, pos, neg) int64. ``rows``: per super-user arrays of positive super-items."""
    n_users = len(rows)
    u = rs.randint(0, n_users, size=(batch,), dtype=np.int64)
    pos = np.empty(batch, np.int64)
    neg = np.empty(batch, np.int64)
    for s in range(batch):
        who = int(u[s])
        attempt = 0
        while attempt < 50 and not (0 < len(rows[who]) < num_items):
            who = int(rs.randint(0, n_users))
            attempt += 1
        u[s] = who
        lst = rows[who]
        usable = 0 < len(lst) < num_items
        p = int(lst[rs.randint(0, len(lst))]) if len(lst) else int(rs.randint(0, num_items))
        q = int(rs.randint(0, num_items))
        if usable:
            members = set(int(x) for x in lst)
            attempt = 0
            while attempt < 50 and (q in members or q == p):
                q = int(rs.randint(0, num_items))
                attempt += 1
        else:
            while q == p:
                q = int(rs.randint(0, num_items))
        pos[s], neg[s] = p, q
    return u, pos, neg


def recall(user_emb: np.ndarray, item_emb: np.ndarray, tr_indptr, tr_indices, test_u, test_i, k: int,
           max_users: int = 5000, scores=None) -> float:
    """Recall@k over the first max_users sorted test users; scores (optional) replaces U @ I^T."""
    test_u, test_i = np.asarray(test_u, np.int64), np.asarray(test_i, np.int64)
    users = np.unique(test_u)[:max_users]
    if users.size == 0:
        return 0.0
    S = (user_emb[users] @ item_emb.T).astype(np.float32) if scores is None else scores.copy()
    hit = total = 0
    n_items = S.shape[1]
    for r, uu in enumerate(users):
        S[r, tr_indices[tr_indptr[uu]:tr_indptr[uu + 1]]] = np.float32(-1e9)
        top = np.lexsort((np.arange(n_items), -S[r].astype(np.float64)))[:min(k, n_items)]
        truth = set(test_i[test_u == uu].tolist())
        hit += len(truth & set(top.tolist()))
        total += len(truth)
    return hit / max(1, total)


def recall_bounds(user_emb: np.ndarray, item_emb: np.ndarray, tr_indptr, tr_indices, test_u, test_i,
                  k: int, max_users: int = 5000, scores=None, rel_tie: float = 0.0):
    """[min, max] of recall_at_k (:446-497) over every order torch.topk could give equal scores.

    Per user the top k are every item scored above the k-th score s_k plus m of the items scored
    s_k (the boundary group, g items of which h are test items): a tie order can place between
    max(0, m - (g - h)) and min(m, h) test items in those m slots. rel_tie > 0 widens the group to
    scores within rel_tie * |s_k| of s_k, for embeddings that drifted from the reference's by fp32
    rounding (two distinct scores that close can swap between the runs). Returns (lo, hi, groups):
    groups = the number of users whose boundary group holds more than m items (0: the value is
    unique, lo == hi)."""
    test_u, test_i = np.asarray(test_u, np.int64), np.asarray(test_i, np.int64)
    users = np.unique(test_u)[:max_users]
    if users.size == 0:
        return 0.0, 0.0, 0
    S = (user_emb[users] @ item_emb.T).astype(np.float32) if scores is None else scores.copy()
    n_items = S.shape[1]
    lo = hi = total = groups = 0
    for r, uu in enumerate(users):
        S[r, tr_indices[tr_indptr[uu]:tr_indptr[uu + 1]]] = np.float32(-1e9)
        truth = np.zeros(n_items, bool)
        tl = test_i[test_u == uu]
        truth[tl] = True
        total += len(set(tl.tolist()))
        if k >= n_items:
            lo += int(truth.sum())
            hi += int(truth.sum())
            continue
        s = S[r].astype(np.float64)
        sk = np.sort(s)[::-1][k - 1]
        tol = rel_tie * abs(sk)
        above = s > sk + tol
        grp = np.abs(s - sk) <= tol
        m = k - int(above.sum())
        g, h = int(grp.sum()), int((grp & truth).sum())
        ha = int((above & truth).sum())
        lo += ha + max(0, m - (g - h))
        hi += ha + min(m, h)
        groups += g > m
    return lo / max(1, total), hi / max(1, total), groups
