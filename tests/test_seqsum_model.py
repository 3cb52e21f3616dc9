"""CPU model of gdd_seqsum.hip's arithmetic (no GPU): the per-binade advance pairs with the
round-to-even parity carry reproduce the sequential fp32 sum bit for bit. The model walks the same
chunks and makes the same decisions as the kernel (term_adv, compose, the first term that leaves
the binade added in fp32), with a small workgroup so that every branch is exercised on short
arrays; the sequential sum is numpy's float32 cumsum (left to right) and the oracle's C loop."""
import math

import numpy as np
import pytest

from oracle import oracle as O

f32 = np.float32
KTOP, KSAT = 1 << 24, 1 << 26


def binade(s):
    E = (int(np.array(s, f32).view(np.uint32)) >> 23) & 0xFF
    return -126 if E == 0 else E - 127


def term_adv(t, e):
    with np.errstate(over="ignore"):
        v = f32(math.ldexp(float(t), 23 - e))
    if not v < f32(33554432.0):
        return (KSAT, KSAT)
    fl = np.floor(v)
    fr = f32(v - fl)
    q = int(fl)
    if fr < 0.5:
        return (q, q)
    if fr > 0.5:
        return (q + 1, q + 1)
    return (q + (q & 1), q + ((q + 1) & 1))


def compose(f, g):
    a = f[0] + (g[1] if f[0] & 1 else g[0])
    b = f[1] + (g[0] if f[1] & 1 else g[1])
    return (min(a, KSAT), min(b, KSAT))


def adv_at(f, S):
    return f[1] if S & 1 else f[0]


def walk(t, nthr=16, E=4):
    """k_seqsum_walk with nthr threads of E terms (the kernel: 1024 x 4)."""
    n, pos, s = len(t), 0, f32(0)
    while pos < n:
        if not np.isfinite(s) or not all(np.isfinite(x) and x >= 0 for x in t[pos:pos + nthr * E]):
            for x in t[pos:]:
                s = f32(s + x)
            return s
        e = binade(s)
        S0 = int(f32(math.ldexp(float(s), 23 - e)))
        fs = []
        for th in range(nthr):
            f = (0, 0)
            for j in range(E):
                i = pos + th * E + j
                f = compose(f, term_adv(t[i], e) if i < n else (0, 0))
            fs.append(f)
        ex, acc = [], (0, 0)
        for f in fs:
            ex.append(acc)
            acc = compose(acc, f)
        S_end = S0 + adv_at(acc, S0)
        if S_end < KTOP:
            s = f32(math.ldexp(S_end, e - 23))
            pos += nthr * E
            continue
        c = next(th for th in range(nthr)
                 if (S0 + adv_at(ex[th], S0)) + adv_at(fs[th], S0 + adv_at(ex[th], S0)) >= KTOP)
        S = S0 + adv_at(ex[c], S0)
        for j in range(E):
            i = pos + c * E + j
            S2 = S + adv_at(term_adv(t[i], e), S)
            if S2 >= KTOP:
                s = f32(f32(math.ldexp(S, e - 23)) + t[i])
                pos = i + 1
                break
            S = S2
        else:
            raise AssertionError("no term left the binade")
    return s


def cases():
    rng = np.random.default_rng(0)
    yield "uniform", rng.random(3000).astype(f32) * 100
    x = rng.integers(0, 8, 2000).astype(f32)
    x[0] = 2.0 ** 24
    yield "ties_odd", x
    x = (rng.integers(0, 8, 2000) + 0.5).astype(f32)
    x[0] = 2.0 ** 23
    yield "ties_half", x
    x = (rng.integers(0, 8, 2000) * 0.5).astype(f32)
    x[0] = 2.0 ** 23 + 1
    yield "ties_odd_start", x
    yield "subnormal", (rng.integers(0, 5, 2000) * f32(2.0 ** -140)).astype(f32)
    yield "heavy_tail", (np.abs(rng.standard_normal(2000)) ** 8).astype(f32)
    yield "zeros", np.zeros(100, f32)
    x = rng.random(1500).astype(f32)
    x[0] = f32(2.0 ** -120)
    yield "tiny_first", x
    yield "huge", np.concatenate([np.full(50, f32(1e-30)), np.full(500, f32(3)), [f32(3e38)],
                                  np.full(10, f32(1))]).astype(f32)
    yield "overflow", np.full(40, f32(1e38))
    x = rng.random(700).astype(f32)
    x[300] = np.nan
    yield "nan", x


@pytest.mark.parametrize("name,x", list(cases()), ids=[c[0] for c in cases()])
def test_model_equals_sequential(name, x):
    ref = np.cumsum(x, dtype=np.float32)[-1]
    got = walk(x)
    if np.isnan(ref):
        assert np.isnan(got)
    else:
        assert got.view(np.uint32) == ref.view(np.uint32), (name, got, ref)
    o = O.inertia(x)
    assert (np.isnan(o) and np.isnan(ref)) or o.view(np.uint32) == ref.view(np.uint32)
