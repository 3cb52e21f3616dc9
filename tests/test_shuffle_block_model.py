"""CPU model of mt_shuffle_draws_block (csrc/gdd_devrng.hpp, r05): the legacy shuffle's draws behind
RandomState.permutation(n) (numpy/random/mtrand.pyx `_shuffle_raw` + `random_interval`, the path
`MiniBatchKMeans._random_reassign` takes through `random_state.choice(b, replace=False, size=m)`,
sklearn/cluster/_kmeans.py:1660) computed by a whole workgroup: each pass takes 2048 tempered words,
each thread walks its `wpt` consecutive words from a guess of its start count, and a block scan of
the per-thread counts is iterated until no count changes (Jacobi). The model follows the kernel's
arithmetic step for step (first guess, change detection, pass bookkeeping) and must give the
sequential draws and the same number of words consumed; numpy itself pins the sequential form."""
import numpy as np
import pytest


def mask32(x):
    x = np.asarray(x, np.int64)
    m = x.copy()
    for s in (1, 2, 4, 8, 16):
        m |= m >> s
    return m


def sequential(words, n):
    """random_interval(i) for i = n-1 .. 1, one word at a time: J and the words consumed."""
    J = np.zeros(n, np.int64)
    i, u = n - 1, 0
    while i >= 1:
        v = int(words[u]) & int(mask32(i))
        u += 1
        if v <= i:
            J[i] = v
            i -= 1
    return J, u


def block_model(words, n, nthreads=1024):
    """mt_shuffle_draws_block: J, words consumed, Jacobi iterations per pass."""
    wpt = 2048 // nthreads
    J = np.zeros(n, np.int64)
    i, start, iters = n - 1, 0, []
    consumed = 0
    tid = np.arange(nthreads)
    while i >= 1:
        w = np.asarray(words[start:start + 2048], np.int64).reshape(nthreads, wpt)
        A = np.minimum(i, (3 * wpt * tid) // 4)
        prev = np.full(nthreads, -1)
        it = 0
        while True:
            it += 1
            a = A.copy()
            fl = np.zeros((nthreads, wpt), bool)
            for u in range(wpt):
                q = i - a
                ok = (q >= 1) & ((w[:, u] & mask32(np.maximum(q, 1))) <= q)
                fl[:, u] = ok
                a += ok
            cnt = a - A
            changed = bool((cnt != prev).any())  # the kernel ORs one flag per wave: the same
            tot = int(cnt.sum())
            prev = cnt
            if not changed:
                break
            A = np.concatenate([[0], np.cumsum(cnt)[:-1]])
        iters.append(it)
        a = A.copy()
        last = None
        for u in range(wpt):
            q = i - a
            sel = fl[:, u]
            J[q[sel]] = w[sel, u] & mask32(q[sel])
            if (sel & (q == 1)).any():
                last = start + wpt * int(np.flatnonzero(sel & (q == 1))[0]) + u
            a += sel
        if tot >= i:
            consumed = last + 1
            i = 0
        else:
            i -= tot
            start += 2048
            consumed = start
    return J, consumed, iters


def tempered_words(seed, count):
    # full-range uint32 randint returns the raw tempered MT19937 words, one per draw
    return np.random.RandomState(seed).randint(0, 2**32, size=count, dtype=np.uint32)


def test_sequential_form_matches_numpy():
    for n, seed in [(2, 0), (10, 1), (1000, 15), (257, 3)]:
        words = tempered_words(seed, 8 * n + 64)
        J, used = sequential(words, n)
        rs = np.random.RandomState(seed)
        pos0 = rs.get_state()[2]
        perm = rs.permutation(n)
        ref = np.arange(n)
        for i in range(n - 1, 0, -1):  # apply the draws as the legacy shuffle does
            ref[i], ref[J[i]] = ref[J[i]], ref[i]
        assert np.array_equal(ref, perm)
        # numpy's position after the shuffle: the words consumed, modulo the 624-word key blocks
        assert rs.get_state()[2] == (pos0 + used - 1) % 624 + 1


@pytest.mark.parametrize("nthreads", [1024, 512, 256])
@pytest.mark.parametrize("n", [2, 3, 64, 65, 1000, 1023, 1024, 1025, 3000, 6000])
def test_block_model_matches_sequential(n, nthreads):
    for seed in range(3):
        words = tempered_words(1000 * n + seed, 8 * n + 4096)
        J, used = sequential(words, n)
        Jb, used_b, iters = block_model(words, n, nthreads)
        assert np.array_equal(J[1:], Jb[1:]) and used == used_b, (n, seed)
        assert max(iters) <= nthreads + 1


def test_block_model_iteration_count_at_batch_1000():
    iters = [max(block_model(tempered_words(s, 12000), 1000)[2]) for s in range(10)]
    assert max(iters) < 64, iters
