"""Drop-in for ``ClustGDD/train_clustgdd_induct.py``: the same flags (and defaults — note
``--sp_ratio 1.0`` and ``--epochs``, which differ from the transductive CLI), seeds and agent flow,
with the inductive agent on libgdd (:class:`gdd.agent_induct.ClustGDD`).

    python -m gdd.train_clustgdd_induct --dataset reddit --reduction_rate 0.005 --prop_num 20 \
        --postprop_num 10 --alpha 0.95 --predropout 0.6 --sp_ratio 0.1 --preep 1000 --postep 1000 \
        --frcoe 0.8 --predcoe 0.05 --w1 0.01 --data_dir data/reddit   (ClustGDD/main_induct.sh)

Datasets: flickr / reddit / ogbn-arxiv load from a GraphSAINT-format directory (``--data_dir``,
default ``data/<dataset>`` as utils_graphsaint.py:17) through :func:`gdd.pipeline.load_graphsaint`;
any other name, or a missing directory, uses the synthetic stand-in of the dataset's shape
(:func:`gdd.data.synthetic`, split into role sub-graphs as ``utils.Transd2Ind``). ``--json`` writes
the accuracies and timings as one JSON line. The reference picks ``cuda`` when available and the
CPU otherwise; this driver needs the MI355X (libgdd has no CPU path).
"""
from __future__ import annotations

import argparse
import json
import os
import random

import numpy as np
import torch

from .train_clustgdd_transduct import parser as _transduct_parser


def parser():
    p = _transduct_parser()
    p.add_argument("--epochs", type=int, default=2000)
    p.set_defaults(sp_ratio=1.0)
    return p


def load_data(args):
    from . import data as D
    saint = ("flickr", "reddit", "ogbn-arxiv")
    path = args.data_dir or os.path.join("data", args.dataset)
    if args.dataset in saint and os.path.exists(os.path.join(path, "adj_full.npz")):
        from .pipeline import load_graphsaint
        return load_graphsaint(path, args.dataset, device=args.device)
    if args.data_dir:
        raise FileNotFoundError(f"no GraphSAINT-format dataset in {args.data_dir}")
    return D.synthetic(args.dataset, seed=args.seed)


def main(argv=None):
    args = parser().parse_args(argv)
    args.device = args.device or "cuda:{}".format(args.gpu_id)
    if torch.device(args.device).type == "cuda":
        torch.cuda.set_device(torch.device(args.device))
    random.seed(args.seed)
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(args.seed)
    print(args)
    data = load_data(args)
    from .agent_induct import ClustGDD
    agent = ClustGDD(data, args, device=args.device)
    out = agent.train()
    if args.json:
        res = agent.results
        with open(args.json, "w") as f:
            json.dump({"dataset": args.dataset, "nodes": int(data.feat_full.shape[0]),
                       "train_nodes": int(data.feat_train.shape[0]), "nnodes_syn": agent.nnodes_syn,
                       "train_test_mean": None if res is None else res.mean(0).tolist(),
                       "train_test_std": None if res is None else res.std(0).tolist(),
                       "runs": None if res is None else res.tolist()}, f)
    return agent, out


if __name__ == "__main__":
    main()
