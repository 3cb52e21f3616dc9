"""CPU model of gdd_kmeanspp.hip's exact parallel sgemv_t lane chains (par_chain_lanes /
par_chain_walk, r05; no GPU): a unit-weight chain acc = acc + x is split into a serial head and
segments whose runs inside one binade are evaluated from 2^e and 2^e + u and composed by parity,
the entries where the sum may change binade added from the exact value. The model makes the kernel's
decisions (fp32 prefix guesses, 2^-9 margins, segmented scan, the walk's checks and the serial
fallback) on numpy float32 scalars; its result must equal the sequential fp32 loop bit for bit."""
import numpy as np
import pytest

f32 = np.float32
ID_E, BAD_E = -1, -2


def bits(v):
    return int(np.array(v, f32).view(np.int32))


def fbits(b):
    return np.array(b, np.int32).view(f32)[()]


def compose(A, B):
    if A[0] == ID_E:
        return B
    if B[0] == ID_E:
        return A
    if A[0] != B[0]:
        return (BAD_E, 0, 0)
    return (A[0], A[1] + (B[2] if A[1] & 1 else B[1]), A[2] + (B[1] if A[2] & 1 else B[2]))


def apply(T, s):
    if T[0] == ID_E:
        return True, s
    bs = bits(s)
    if (bs >> 23) != T[0]:
        return False, s
    nb = bs + (T[2] if bs & 1 else T[1])
    if (nb >> 23) != T[0]:
        return False, s
    return True, fbits(nb)


def seq(x, acc0):
    s = f32(acc0)
    for v in x:
        s = f32(s + f32(v))
    return s


def par_chain(xc, acc0, G=32, H=32, MS=16, stats=None):
    xc = [f32(v) for v in xc]
    L = len(xc)
    Hh = min(H, L)
    seg = min(MS, (((L - Hh + G - 1) // G) + 3) & ~3)
    lanes = []
    for g in range(G):
        a = Hh + g * seg
        cnt = max(0, min(seg, L - a))
        x = [xc[a + i] if i < cnt else f32(0) for i in range(MS)]
        loc, run = [], f32(0)
        for v in x:
            run = f32(run + v)
            loc.append(run)
        lanes.append(dict(a=a, cnt=cnt, x=x, loc=loc, run=run, hx=xc[g] if g < Hh else f32(0)))
    inc = [ln["run"] for ln in lanes]
    hx = [ln["hx"] for ln in lanes]
    o = 1
    while o < G:  # Kogge-Stone (all lanes read the previous step's values)
        inc = [f32(inc[g] + inc[g - o]) if g >= o else inc[g] for g in range(G)]
        hx = [f32(hx[g] + hx[g ^ o]) for g in range(G)]
        o <<= 1
    kLo, kHi = f32(1.0 - 1.0 / 512), f32(1.0 + 1.0 / 512)
    elems = []
    for g, ln in enumerate(lanes):
        ps = f32(f32(f32(acc0) + hx[g]) + f32(inc[g] - ln["run"]))
        cnt, loc, x = ln["cnt"], ln["loc"], ln["x"]
        cm = 0
        for i in range(MS):
            prev = f32(ps + loc[i - 1]) if i else ps
            cur = f32(ps + loc[i])
            el, eh = bits(f32(prev * kLo)) >> 23, bits(f32(cur * kHi)) >> 23
            if i < cnt and not (el == eh and el >= 1 and eh <= 253):
                cm |= 1 << i
        j1 = (cm & -cm).bit_length() - 1 if cm else cnt
        j2 = cm.bit_length() - 1 if cm else cnt - 1
        kind = 0 if cm == 0 else (1 if (cm >> j1) == (2 << (j2 - j1)) - 1 else 2)
        eA = bits(ps) >> 23 if j1 > 0 else 127
        eB = bits(f32(ps + loc[cnt - 1])) >> 23 if (kind == 1 and j2 < cnt - 1) else 127
        a0, a1 = fbits(eA << 23), fbits((eA << 23) + 1)
        b0, b1 = fbits(eB << 23), fbits((eB << 23) + 1)
        for i in range(MS):
            xa = x[i] if i < j1 else f32(0)
            xb = x[i] if (j2 < i < cnt) else f32(0)
            a0, a1, b0, b1 = f32(a0 + xa), f32(a1 + xa), f32(b0 + xb), f32(b1 + xb)
        A = (eA, bits(a0) - (eA << 23), bits(a1) - (eA << 23) - 1) if j1 > 0 else (ID_E, 0, 0)
        hasB = kind == 1 and j2 < cnt - 1
        B = (eB, bits(b0) - (eB << 23), bits(b1) - (eB << 23) - 1) if hasB else (ID_E, 0, 0)
        if (j1 > 0 and (bits(a1) >> 23) != eA) or (hasB and (bits(b1) >> 23) != eB):
            kind = 2
        f = int(kind != 0)
        T = A if kind == 0 else (B if kind == 1 else (ID_E, 0, 0))
        x0 = ln["a"] if kind == 2 else ln["a"] + j1
        x1 = ln["a"] + cnt if kind == 2 else (ln["a"] + j2 + 1 if kind == 1 else ln["a"] + j1)
        elems.append(dict(f=f, T=T, A=A, kind=kind, x0=x0, x1=x1))
        if stats is not None:
            stats[kind] = stats.get(kind, 0) + 1
    fs, Ts = [e["f"] for e in elems], [e["T"] for e in elems]
    o = 1
    while o < G:  # segmented inclusive scan
        nf, nT = list(fs), list(Ts)
        for g in range(o, G):
            if not fs[g]:
                nT[g] = compose(Ts[g - o], Ts[g])
                nf[g] = fs[g - o]
        fs, Ts, o = nf, nT, o * 2
    # the walker: head serially, then the crossing segments
    s = seq(xc[:Hh], acc0)
    ok = True
    for q in range(G):
        e = elems[q]
        if e["kind"] == 0:
            continue
        if q > 0:
            r, s = apply(Ts[q - 1], s)
            ok = ok and r
        if e["kind"] == 1:
            r, s = apply(e["A"], s)
            ok = ok and r
        for i in range(e["x0"], e["x1"]):
            s = f32(s + xc[i])
    r, s = apply(Ts[G - 1], s)
    ok = ok and r
    if stats is not None:
        stats["fallback"] = stats.get("fallback", 0) + (not ok)
    return s if ok else seq(xc, acc0)


def cases():
    rng = np.random.default_rng(0)
    out = []
    for L in (0, 1, 5, 31, 32, 33, 100, 375, 512):
        out.append(("uniform", rng.uniform(0, 1, L).astype(f32)))
    out.append(("integers", rng.integers(0, 5000, 375).astype(f32)))  # sums past 2^24: ties
    out.append(("int_small", rng.integers(0, 3, 512).astype(f32) * f32(2 ** 20)))
    z = rng.uniform(0, 1, 375).astype(f32)
    z[::3] = 0
    z[40:200] = 0
    out.append(("zeros", z))
    out.append(("decades", (10.0 ** rng.uniform(-12, 12, 375)).astype(f32)))
    big = rng.uniform(0, 1e-6, 375).astype(f32)
    big[0] = 1e6
    out.append(("absorbed", big))
    out.append(("all_zero", np.zeros(375, f32)))
    sub = np.full(375, 1e-40, f32)
    out.append(("subnormal", sub))
    inf = rng.uniform(0, 1, 375).astype(f32)
    inf[200] = np.inf
    out.append(("inf", inf))
    grow = (np.arange(375, dtype=np.float64) ** 3).astype(f32)
    out.append(("growing", grow))
    return out


@pytest.mark.parametrize("name,x", cases(), ids=[c[0] + str(len(c[1])) for c in cases()])
@pytest.mark.parametrize("acc0", [0.0, 0.75])
@pytest.mark.parametrize("G", [32, 64])
def test_par_chain_model_matches_sequential(name, x, acc0, G):
    ref = seq(x, acc0)
    got = par_chain(x, acc0, G=G)
    assert bits(got) == bits(ref) or (np.isnan(got) and np.isnan(ref))


def test_par_chain_model_ties_exercised():
    """The integer chain's sums pass 2^24, so quanta exceed 1 and exact ties occur: the parity
    composition (not the fallback) gives the sequential bits."""
    rng = np.random.default_rng(5)
    stats = {}
    for _ in range(20):
        x = rng.integers(0, 20000, 375).astype(f32)
        assert bits(par_chain(x, 0.0, stats=stats)) == bits(seq(x, 0.0))
    assert stats.get("fallback", 0) == 0 and stats.get(0, 0) > 0
