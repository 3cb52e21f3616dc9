"""Drop-in for ``ClustGDD/train_clustgdd_transduct.py``: the same flags (and defaults), seeds and
agent flow, with the agent on libgdd (:class:`gdd.agent.ClustGDD`).

    python -m gdd.train_clustgdd_transduct --dataset ogbn-arxiv --reduction_rate 0.005 \
        --prop_num 18 --alpha 0.91 ...   (ClustGDD/main_transduct.sh's settings)

Datasets: a GraphSAINT-format directory (``--data_dir``; ``adj_full.npz``, ``role.json``,
``feats.npy``, ``class_map.json``, as utils_graphsaint.DataGraphSAINT reads) when given, otherwise
the synthetic stand-in of the dataset's shape (:func:`gdd.data.synthetic`; the Planetoid / OGB
downloads the reference performs are unavailable offline). ``--json`` writes the distilled-graph
accuracy and timings as one JSON line.
"""
from __future__ import annotations

import argparse
import json
import random

import numpy as np
import torch


def parser():
    p = argparse.ArgumentParser()
    p.add_argument("--gpu_id", type=int, default=0, help="gpu id")
    p.add_argument("--dataset", type=str, default="cora")
    p.add_argument("--nlayers", type=int, default=2)
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--weight_decay", type=float, default=0.0)
    p.add_argument("--dropout", type=float, default=0.0)
    p.add_argument("--normalize_features", type=bool, default=True)
    p.add_argument("--keep_ratio", type=float, default=1.0)
    p.add_argument("--reduction_rate", type=float, default=1)
    p.add_argument("--seed", type=int, default=15, help="Random seed.")
    p.add_argument("--sgc", type=int, default=1)
    p.add_argument("--save", type=int, default=0)
    p.add_argument("--gctype", type=str, default="clustgdd")
    p.add_argument("--prop_num", type=int, default=1, help="the steps of feature propagations")
    p.add_argument("--alpha", type=float, default=0.8, help="the prop coe")
    p.add_argument("--prehidden", type=int, default=256)
    p.add_argument("--predropout", type=float, default=0.6)
    p.add_argument("--prewd", type=float, default=5e-4)
    p.add_argument("--prelr", type=float, default=0.01)
    p.add_argument("--preep", type=int, default=600, help="pretraining epochs")
    p.add_argument("--prenlayers", type=int, default=2)
    p.add_argument("--cluster_minibatch", type=int, default=1000)
    p.add_argument("--sp_ratio", type=float, default=0.05)
    p.add_argument("--sp_type", type=str, default="attaw")
    p.add_argument("--postep", type=int, default=100)
    p.add_argument("--postprop_num", type=int, default=1)
    p.add_argument("--postlr_feat", type=float, default=1e-4)
    p.add_argument("--postlr_adj", type=float, default=1e-4)
    p.add_argument("--postlr_model", type=float, default=1e-2)
    p.add_argument("--postwd_feat", type=float, default=5e-4)
    p.add_argument("--postwd_adj", type=float, default=5e-4)
    p.add_argument("--postwd_model", type=float, default=5e-4)
    p.add_argument("--frcoe", type=float, default=0.01)
    p.add_argument("--predcoe", type=float, default=1.0)
    p.add_argument("--csttemp", type=float, default=0.5)
    p.add_argument("--w1", type=float, default=0.1)
    p.add_argument("--w2", type=float, default=1.0)
    p.add_argument("--no_refinement", type=bool, default=False)
    p.add_argument("--no_adjsyn", type=bool, default=False)
    p.add_argument("--save_pretrained_output", type=bool, default=False)
    p.add_argument("--save_syn_output", type=bool, default=False)
    p.add_argument("--save_norf", type=bool, default=False)
    p.add_argument("--notopo", type=bool, default=False)
    p.add_argument("--tm_rec", type=bool, default=False)
    # gdd additions
    p.add_argument("--data_dir", type=str, default="", help="GraphSAINT-format dataset directory")
    p.add_argument("--device", type=str, default="", help="cuda:<gpu_id> by default")
    p.add_argument("--json", type=str, default="", help="write accuracy + timings as JSON here")
    return p


def load_data(args):
    from . import data as D
    if args.data_dir:
        from .pipeline import load_graphsaint
        ns = load_graphsaint(args.data_dir, args.dataset, device=args.device)
        return D.Transd2Ind(ns.adj_full.to_scipy(), ns.feat_full.cpu().numpy(), ns.labels_full,
                            ns.idx_train.cpu().numpy(), ns.idx_val.cpu().numpy(), ns.idx_test.cpu().numpy())
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
    from .agent import ClustGDD
    agent = ClustGDD(data, args, device=args.device)
    agent.train()
    if args.json:
        res = agent.results
        with open(args.json, "w") as f:
            json.dump({"dataset": args.dataset, "nodes": int(data.feat_full.shape[0]),
                       "nnodes_syn": agent.nnodes_syn,
                       "train_test_mean": None if res is None else res.mean(0).tolist(),
                       "train_test_std": None if res is None else res.std(0).tolist(),
                       "runs": None if res is None else res.tolist()}, f)
    return agent


if __name__ == "__main__":
    main()
