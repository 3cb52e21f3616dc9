"""Host-side pieces of the k-means drop-ins that must consume a RandomState exactly as scikit-learn does."""
import numpy as np
import pytest

from gdd.kmeans import choice_unit_weights


@pytest.mark.parametrize("n", [1, 2, 3, 7, 1000, 3000, 6040, 65537, 169343, 2449029])
def test_choice_unit_weights_matches_numpy(n):
    """sklearn's first k-means++ centre, rs.choice(n, p=w / w.sum()) with unit float32 weights: same
    index and same generator state afterwards, without the O(n) arrays."""
    w = np.ones(n, dtype=np.float32)
    seeds = range(40) if n < 100000 else range(6)
    for seed in seeds:
        a, b = np.random.RandomState(seed), np.random.RandomState(seed)
        ref = int(a.choice(n, p=w / w.sum()))
        got = choice_unit_weights(b, n)
        assert got == ref, (n, seed)
        sa, sb = a.get_state(), b.get_state()
        assert np.array_equal(sa[1], sb[1]) and sa[2] == sb[2]


def test_choice_unit_weights_edges():
    # uniforms at the cdf steps: u = k / n exactly and its neighbours
    n = 6040
    w = np.ones(n, dtype=np.float32)
    p = w / w.sum()
    cdf = np.cumsum(p.astype(np.float64))
    cdf /= cdf[-1]

    class Fixed:
        def __init__(self, u):
            self.u = u

        def random_sample(self):
            return self.u

    for k in (1, 17, 3020, 6039):
        for u in (np.nextafter(k / n, 0), k / n, np.nextafter(k / n, 1)):
            assert choice_unit_weights(Fixed(float(u)), n) == int(np.searchsorted(cdf, u, side="right"))


@pytest.mark.parametrize("seed", [0, 15, 42])
@pytest.mark.parametrize("k,T", [(2, 2), (454, 8), (604, 8), (1773, 9)])
def test_kpp_uniforms_in_one_draw(seed, k, T):
    """_kmeans_plusplus draws random_state.uniform(size=n_local_trials) once per round
    (sklearn/cluster/_kmeans.py:247); _Ops.kmeans_plusplus draws all (k - 1) * T at once. The legacy
    RandomState stream gives the same doubles, and leaves the generator in the same state."""
    a, b = np.random.RandomState(seed), np.random.RandomState(seed)
    a.random_sample()
    b.random_sample()  # the first centre's draw
    u_rounds = np.concatenate([a.uniform(size=T) for _ in range(k - 1)])
    u_once = b.uniform(size=(k - 1) * T)
    assert np.array_equal(u_rounds.view(np.int64), u_once.view(np.int64))
    sa, sb = a.get_state(), b.get_state()
    assert np.array_equal(sa[1], sb[1]) and sa[2:] == sb[2:]
