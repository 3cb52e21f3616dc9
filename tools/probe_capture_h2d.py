#!/usr/bin/env python3
"""What a HIP-graph-captured host-to-device copy of a pageable numpy array reads at replay — the
suspected cause of r03's captured recsys epoch faulting on its first replay at the Ali-Display shape
(VERDICT r3 #4): the epoch copied the host-sampled BPR triplets (`torch.from_numpy(u).to(dev)`) inside
the capture. No kernel consumes the copied values here, so a stale read cannot fault the GPU.

Prints, for a 4,096-entry int64 array (the Ali-Display batch) and a 256-entry one (the small fixture):
whether capture succeeded, whether a replay sees the array's current contents (the node re-reads the
capture-time host address) and what it reads after the array is freed and other arrays are allocated."""
import gc

import numpy as np
import torch


def probe(b):
    dev = torch.device("cuda")
    a = np.arange(b, dtype=np.int64)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        d = torch.from_numpy(a).to(dev)  # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    try:
        with torch.cuda.graph(g):
            d = torch.from_numpy(a).to(dev)
    except Exception as e:  # noqa: BLE001
        print(f"b={b}: capture refused: {type(e).__name__}: {str(e).splitlines()[0]}", flush=True)
        return
    torch.cuda.synchronize()
    a[:] = 7
    g.replay()
    torch.cuda.synchronize()
    live = bool((d.cpu().numpy() == 7).all())
    first = d.cpu().numpy()[:4].tolist()
    addr = a.ctypes.data
    del a
    gc.collect()
    junk = [np.full(b, -123456789, np.int64) for _ in range(8)]  # reuse the freed block
    reused = any(j.ctypes.data == addr for j in junk)
    g.replay()
    torch.cuda.synchronize()
    after = d.cpu().numpy()
    in_range = bool(((after >= 0) & (after < b)).all())
    print(f"b={b}: replay reads the array's current contents: {live} (first {first}); after free + "
          f"8 new arrays (one at the old address: {reused}): values in [0, b): {in_range}, "
          f"first {after[:4].tolist()}", flush=True)
    del junk


def main():
    for b in (256, 4096, 4096 * 3):
        probe(b)


if __name__ == "__main__":
    main()
