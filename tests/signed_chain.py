"""CPU model of an exact parallel fp32 chain sum (test infrastructure: imported by tests/ and
tools/model_lloyd_rank_split.py; never by the product path). A sequential fp32 sum of SIGNED terms — numpy's column sums
(csrc/gdd_colsum.hip, r05) and sklearn's Lloyd M-step per (cluster, column) chain
(_k_means_lloyd.pyx:140-152, one thread) — evaluated from per-segment two-state transducers:
while the running sum s stays in one signed binade (sign sigma, |s| in [2^e, 2^(e+1))), s = S*u with
u = 2^(e-23) and S a signed integer; a term t moves S by round(t/u), ties to the even S — an advance
that depends only on S's parity. A run of terms is then a transducer (per start parity: the advance,
and the least and greatest partial advance), runs compose associatively, and the composed run applies
exactly when its path stays strictly inside the binade (one unit of margin at the edge nearer zero,
where the grid halves).

rank_split_fold (r06) models the multi-GPU form of the Lloyd M-step fold: each rank
holds a contiguous block of a chain's terms (its rows' members), cuts it into segments, and ships per
segment either transducer records for two candidate binades (from an fp64 estimate of the global
prefix: one all-gather of per-rank fp64 totals) or — where its fp64 path comes near a binade edge —
the raw terms; a resolver composes the segments in rank order from +0 and either reproduces the
sequential sum bit for bit or reports that a record did not apply (the iteration then falls back to
the labels all-gather)."""
import numpy as np

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


def rank_split_fold(blocks, L=256, eps=2.0 ** -10):
    """The rank-split fold of one chain. blocks: the ranks' term arrays (float32, in rank order).
    Returns (s, stats): s the fp32 sum (None if a shipped record did not apply: the fallback), stats
    the shipped volume (records, raw terms) and the segment counts."""
    segs = []  # (rank, terms)
    for r, b in enumerate(blocks):
        b = np.asarray(b, np.float32)
        for i in range(0, len(b), L):
            segs.append((r, b[i:i + L]))
    # collective A: the per-rank fp64 totals (a prefix over ranks); within a rank, the segments' sums
    totals = [float(np.sum(np.asarray(b, np.float64))) for b in blocks]
    pre_rank = np.concatenate([[0.0], np.cumsum(totals)])[:-1]
    ship = []
    nrec = nraw = 0
    run = {r: pre_rank[r] for r in range(len(blocks))}
    for r, t in segs:
        P = run[r]
        path = P + np.cumsum(t.astype(np.float64))
        run[r] = float(path[-1]) if len(t) else P
        allp = np.concatenate([[P], path])
        fin = np.isfinite(allp).all() and np.isfinite(t).all()
        risky = not fin
        if not risky:
            a = np.abs(allp)
            if (a == 0).any() or (np.sign(allp) != np.sign(allp[0])).any():
                risky = True
            else:
                ex = np.floor(np.log2(a))
                if (ex != ex[0]).any():
                    risky = True  # the fp64 path crosses a binade edge
                else:
                    rel_lo = a / np.exp2(ex) - 1.0        # distance to the lower edge (relative)
                    rel_hi = 2.0 - a / np.exp2(ex)        # to the upper edge
                    risky = bool((rel_lo < eps).any() or (rel_hi < eps).any())
        if risky:
            ship.append(("raw", t))
            nraw += 1
        else:
            es = guess(P)
            ship.append(("rec", es, [run_tr(t, e) for e in es]))
            nrec += 1
    # the resolver: every rank, from +0, in rank order
    s = np.float32(0.0)
    for item in ship:
        if item[0] == "raw":
            s = walk(item[1], s)
            continue
        _, es, fs = item
        if not np.isfinite(s):
            return None, {"records": nrec, "raw": nraw, "fallback": True}
        e, S = binade(s)
        done = False
        for ec, f in zip(es, fs):
            if ec == e and applies(S, e, f):
                s = np.float32(np.ldexp(np.float64(S + f[S & 1][0]), e - 23))
                done = True
                break
        if not done:
            return None, {"records": nrec, "raw": nraw, "fallback": True}
    return s, {"records": nrec, "raw": nraw, "fallback": False}
