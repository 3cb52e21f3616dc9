#!/usr/bin/env python3
"""How does eager `t / python_float` round on this torch build (true division, or multiplication by an
fp32 reciprocal)? The graph-captured Adam step of gdd.distill_recsys must reproduce it bit for bit."""
import numpy as np
import torch

t = torch.randn(1 << 20, device="cuda") * 10
ok_div = ok_mul = 0
for step in range(1, 200):
    c = 1 - 0.999 ** step
    eager = (t / c).cpu().numpy()
    true_div = (t / torch.tensor(c, dtype=torch.float32, device="cuda")).cpu().numpy()
    recip = (t * torch.tensor(np.float32(1.0) / np.float32(c), device="cuda")).cpu().numpy()
    ok_div += np.array_equal(eager.view(np.uint32), true_div.view(np.uint32))
    ok_mul += np.array_equal(eager.view(np.uint32), recip.view(np.uint32))
print(f"eager t / c equals: true fp32 division in {ok_div}/199 steps, x fp32(1/c) in {ok_mul}/199 steps")
