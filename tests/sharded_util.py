"""Test helpers for gdd.sharded: a CPU stand-in for the device primitives (the oracle's arithmetic,
test-only) and a gloo process-group runner."""
import os
import socket

import numpy as np
import torch

from oracle import oracle as O


class OracleOps:
    """The five primitives ShardedKMeans needs, computed by the oracle on the host."""

    device = torch.device("cpu")

    def tensor(self, a, dtype=None):
        return torch.as_tensor(a, dtype=dtype)

    def assign(self, X, C, labels, sq):
        lab, s = O.assign(X.numpy(), C.numpy())
        labels.copy_(torch.from_numpy(lab))
        sq.copy_(torch.from_numpy(s))

    def segment_sum_fixed(self, X, labels, k, scale_exp):
        v = np.rint(X.numpy().astype(np.float64) * (2.0 ** scale_exp)).astype(np.int64)
        sums = np.zeros((k, X.shape[1]), np.int64)
        np.add.at(sums, labels.numpy(), v)
        counts = np.bincount(labels.numpy(), minlength=k).astype(np.int64)
        return torch.from_numpy(sums), torch.from_numpy(counts)

    def fixed_to_centers(self, sums, counts, scale_exp, C):
        s, c = sums.numpy().astype(np.float64), counts.numpy()
        m = c > 0
        vals = ((s * (2.0 ** -scale_exp))[m] / c[m, None]).astype(np.float32)
        Cn = C.numpy()
        Cn[m] = vals

    def kmeans_plusplus(self, X, k, rs):
        centers, _ = O.kmeans_plusplus(X.numpy(), k, rs)
        return torch.from_numpy(centers)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def init_gloo(rank, world, port):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
