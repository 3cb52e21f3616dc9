"""CPU model of the exact parallel form of a sequential fp32 sum of SIGNED terms (csrc/gdd_colsum.hip,
r05): numpy's column sums of a C-contiguous float32 matrix (`X.mean(axis=0)`, `X.var(axis=0)` in
KMeans.fit's centring and _tolerance, sklearn/cluster/_kmeans.py:1476-1487 and :279-288) are one
sequential fp32 chain per column. While the running sum s stays in one signed binade (sign sigma,
|s| in [2^e, 2^(e+1))), s = S*u with u = 2^(e-23) and S a signed integer; a term t moves S by
round(t/u), ties to the even S — an advance that depends only on S's parity. A run of terms is then a
two-state transducer (per start parity: the advance, and the least and greatest partial advance), runs
compose associatively, and the composed run applies exactly when its path stays strictly inside the
binade (one unit of margin at the edge nearer zero, where the grid halves). The model follows the
kernels' arithmetic (candidate binades from an fp64 prefix, per-segment transducers, a resolve that
re-walks a segment whose transducer does not apply) and must give the sequential sum bit for bit."""
import numpy as np
import pytest

SAT = 1 << 27
TOP = 1 << 24
LOW = 1 << 23


def sat(x):
    return max(-SAT, min(SAT, x))


def binade(s):
    """(e, S) of a finite fp32 s: e = -126 for |s| < 2^-125 (subnormals share binade -126's grid)."""
    s = np.float32(s)
    E = (int(s.view(np.uint32)) >> 23) & 0xFF
    e = -126 if E <= 1 else E - 127
    S = int(np.ldexp(np.float64(s), 23 - e))  # exact: s is a multiple of u
    return e, S


def term_tr(t, e):
    """the transducer of one term in binade e: {parity: (advance, min, max)}"""
    v = np.ldexp(np.float64(np.float32(t)), 23 - e)  # exact (t/u is a dyadic of <= 24 bits)
    if not abs(v) < 2.0 ** 26:
        q0 = q1 = SAT if v > 0 else -SAT
    else:
        fl = np.floor(v)
        fr = v - fl
        q = int(fl)
        if fr < 0.5:
            q0 = q1 = q
        elif fr > 0.5:
            q0 = q1 = q + 1
        else:  # tie: the even one of S+q, S+q+1
            q0 = q + (q & 1)
            q1 = q + ((q + 1) & 1)
    return {0: (q0, q0, q0), 1: (q1, q1, q1)}


# the empty run: no partial sums, so its least partial advance is +SAT and its greatest -SAT (a start
# exactly on the binade's lower edge is not itself a violation)
IDENT = {0: (0, SAT, -SAT), 1: (0, SAT, -SAT)}


def compose(f, g):
    out = {}
    for p in (0, 1):
        a, mn, mx = f[p]
        p2 = (p + a) & 1
        b, mn2, mx2 = g[p2]
        out[p] = (sat(a + b), min(mn, sat(a + mn2)), max(mx, sat(a + mx2)))
    return out


def applies(S0, e, f):
    """the run applies from S0 (binade e, S0 inside it): every partial sum stays strictly inside"""
    a, mn, mx = f[S0 & 1]
    lo, hi = S0 + mn, S0 + mx
    if e == -126:  # one grid from -2^-125 to 2^-125, zero included
        return -TOP < lo and hi < TOP
    if S0 > 0:
        return lo > LOW and hi < TOP
    return hi < -LOW and lo > -TOP


def seq_sum(t, s=np.float32(0.0)):
    s = np.float32(s)
    for x in t:
        s = np.float32(s + np.float32(x))
    return s


def run_tr(t, e):
    f = IDENT
    for x in t:
        f = compose(f, term_tr(x, e))
    return f


def walk(t, s):
    """the chunked walk: scan a chunk's composed path; where it stops applying, add that term in
    hardware and resume after it (the model walks term by term inside the failing chunk)"""
    s = np.float32(s)
    i = 0
    while i < len(t):
        if not np.isfinite(s) or not np.isfinite(t[i]):
            return seq_sum(t[i:], s)
        e, S = binade(s)
        f = term_tr(t[i], e)
        if applies(S, e, f):
            S2 = S + f[S & 1][0]
            s = np.float32(np.ldexp(np.float64(S2), e - 23))
        else:
            s = np.float32(s + np.float32(t[i]))
        i += 1
    return s


def guess(P):
    p = np.float32(P)
    if not np.isfinite(p):  # the segment is re-walked
        return [127, 127]
    e, _ = binade(p)
    if e == -126:
        return [e, -125]
    r = abs(float(np.ldexp(np.float64(p), -e)))
    return [e, min(e + 1, 127) if r >= 1.5 else e - 1]


def segmented(t, L):
    """segments of L terms: fp64 prefixes -> two candidate binades -> transducers -> resolve"""
    n = len(t)
    nseg = (n + L - 1) // L
    segsum = [float(np.sum(t[b * L:(b + 1) * L], dtype=np.float64)) for b in range(nseg)]
    recs = []
    P = 0.0
    for b in range(nseg):
        es = guess(P)
        seg = t[b * L:(b + 1) * L]
        bad = not np.isfinite(seg).all()
        recs.append((es, [run_tr(seg, e) for e in es], bad))
        P += segsum[b]
    s = np.float32(0.0)
    rewalks = 0
    for b in range(nseg):
        es, fs, bad = recs[b]
        seg = t[b * L:(b + 1) * L]
        done = False
        if np.isfinite(s) and not bad:
            e, S = binade(s)
            for ec, f in zip(es, fs):
                if ec == e and applies(S, e, f):
                    s = np.float32(np.ldexp(np.float64(S + f[S & 1][0]), e - 23))
                    done = True
                    break
        if not done:
            rewalks += 1
            s = walk(seg, s)
    return s, rewalks


def cases():
    rng = np.random.default_rng(7)
    yield "zero-mean", rng.standard_normal(3000).astype(np.float32)
    yield "drift", (rng.standard_normal(3000) + 0.3).astype(np.float32)
    yield "negative drift", (rng.standard_normal(3000) - 2.0).astype(np.float32)
    yield "ties", (rng.integers(-4, 5, 3000) * 0.5 + 2 ** 23).astype(np.float32)
    yield "integers past 2^24", rng.integers(-3, 9, 3000).astype(np.float32) * np.float32(4096.0)
    yield "cancel to zero", np.concatenate([np.full(500, 0.1, np.float32), np.full(500, -0.1, np.float32),
                                            rng.standard_normal(1000).astype(np.float32)])
    yield "subnormals", (rng.standard_normal(2000) * 1e-40).astype(np.float32)
    yield "decades", (rng.standard_normal(3000) * 10.0 ** rng.integers(-12, 12, 3000)).astype(np.float32)
    yield "zeros and signed zeros", np.array([0.0, -0.0] * 300 + [1e-3, -1e-3] * 200, np.float32)
    x = rng.standard_normal(2000).astype(np.float32)
    x[777] = np.inf
    yield "infinity", x
    x = rng.standard_normal(2000).astype(np.float32)
    x[1500] = np.nan
    yield "nan", x


@pytest.mark.parametrize("name,t", list(cases()), ids=[c[0] for c in cases()])
@pytest.mark.parametrize("L", [64, 256])
def test_segmented_matches_sequential(name, t, L):
    ref = seq_sum(t)
    got, rewalks = segmented(t, L)
    assert (np.isnan(ref) and np.isnan(got)) or ref.view(np.uint32) == got.view(np.uint32), (name, ref, got)


def test_walk_matches_sequential_term_by_term():
    rng = np.random.default_rng(3)
    for _ in range(20):
        t = (rng.standard_normal(400) * 10.0 ** rng.integers(-3, 4)).astype(np.float32)
        s0 = np.float32(rng.standard_normal() * 10.0 ** rng.integers(-3, 4))
        assert seq_sum(t, s0).view(np.uint32) == walk(t, s0).view(np.uint32)


def test_drifting_sums_rarely_rewalk():
    t = (np.random.default_rng(5).standard_normal(20000) + 1.0).astype(np.float32)
    s, rewalks = segmented(t, 256)
    assert s.view(np.uint32) == seq_sum(t).view(np.uint32)
    assert rewalks <= 20  # the binade changes (~log2 of the sum's range), not every segment
