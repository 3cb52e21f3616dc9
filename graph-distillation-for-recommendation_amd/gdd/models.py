"""The two torch models the ClustGDD agents train around the hot path (out of the kernel scope, but
they produce the k-means input and the downstream metric the BASELINE quotes):

* :class:`MLP` — ``models/gcn.py:440-653`` as the agents use it: a linear (``with_relu=False``)
  2-layer MLP trained ``preep`` epochs on the propagated features with best-validation weights;
  ``predict(x, mode='e')`` gives (log-softmax, logits), and the logits are the k-means input
  (clustgdd_agent_transduct.py:66-100);
* :class:`GCN` — ``models/gcn.py:58-362``: the evaluator trained on the distilled graph for 600
  epochs (LR / 10 at half) with the full graph scored every epoch (``_train_with_val``), as
  ``test_with_val`` runs it five times (transduct:349-393).

Semantics follow the reference exactly — parameter creation order, the double initialisation
(constructor, then ``initialize()``), dropout calls, the Adam restarts and the strict ``>``
best-validation rule — so on the same device and seed the accuracies equal the reference's
(tests/test_agent_cpu.py, fixture G10). The difference is where the products run: a
:class:`gdd.graph.CSRGraph` adjacency goes through libgdd's planned SpMM (``gdd.gcn.spmm``), and
the reference's redundant host re-normalisations of the full graph per ``fit`` are done once on
the device (``normalize_adj``); torch sparse / dense adjacencies keep ``torch.spmm``.
"""
from __future__ import annotations

from copy import deepcopy

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn, optim

from .gcn import GraphConvolution


def accuracy(output: torch.Tensor, labels) -> torch.Tensor:
    """deep_robust_utils.accuracy: share of argmax(output) == labels, as a float64 tensor."""
    if not isinstance(labels, torch.Tensor):
        labels = torch.LongTensor(np.atleast_1d(labels))
    preds = output.max(1)[1].type_as(labels)
    return preds.eq(labels).double().sum() / len(labels)


def normalize_dense(adj: torch.Tensor) -> torch.Tensor:
    """normalize_adj_tensor(adj) for a dense tensor (deep_robust_utils.py:257-264):
    D^-1/2 (A + I) D^-1/2 with inf -> 0, as two diagonal matmuls."""
    mx = adj + torch.eye(adj.shape[0], device=adj.device)
    r = mx.sum(1).pow(-0.5).flatten()
    r[torch.isinf(r)] = 0.0
    d = torch.diag(r)
    return (d @ mx) @ d


def normalize_any(adj):
    """The reference's normalize_adj_tensor dispatch: CSRGraph / torch sparse -> libgdd CSR
    normalisation (sparse=True path), dense -> :func:`normalize_dense`."""
    from .graph import CSRGraph, normalize_adj, to_csr
    if isinstance(adj, CSRGraph):
        return normalize_adj(adj)
    if isinstance(adj, torch.Tensor) and not adj.is_sparse:
        return normalize_dense(adj)
    if isinstance(adj, torch.Tensor) and adj.device.type == "cpu":
        return _normalize_sparse_cpu(adj)
    return normalize_adj(to_csr(adj, device=adj.device if isinstance(adj, torch.Tensor) else "cuda"))


def _normalize_sparse_cpu(adj: torch.Tensor) -> torch.Tensor:
    """The reference's sparse path on the host (scipy in fp64, fp32 COO out) — used when the
    models run on the CPU (tests against the reference's own numbers)."""
    import scipy.sparse as sp
    a = adj.coalesce()
    n = a.shape[0]
    M = sp.csr_matrix((a.values().numpy(), a.indices().numpy()), shape=(n, n)).tolil()
    if M[0, 0] == 0:
        M = M + sp.eye(n)
    with np.errstate(divide="ignore"):
        r = np.power(np.array(M.sum(1)), -0.5).flatten()
    r[np.isinf(r)] = 0.0
    D = sp.diags(r)
    M = D.dot(M).dot(D).tocoo().astype(np.float32)
    idx = torch.from_numpy(np.vstack((M.row, M.col)).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(M.data), (n, n))


def _as_device_graph(adj, device):
    """A full-graph adjacency for the per-epoch evaluation: CSRGraph stays, scipy / torch sparse
    become a CSRGraph on a GPU device and a torch sparse tensor on the CPU."""
    from .graph import CSRGraph, to_csr
    if isinstance(adj, CSRGraph):
        return adj
    dev = torch.device(device)
    if dev.type == "cuda":
        return to_csr(adj, device=dev)
    if isinstance(adj, torch.Tensor):
        return adj.to(dev)
    import scipy.sparse as sp
    m = sp.coo_matrix(adj).astype(np.float32)
    idx = torch.from_numpy(np.vstack((m.row, m.col)).astype(np.int64))
    return torch.sparse_coo_tensor(idx, torch.from_numpy(m.data), m.shape)


def _feat(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device)
    return torch.FloatTensor(np.array(x)).to(device)


class _Trainable(nn.Module):
    """Shared layer stack and the best-validation training loop of models/gcn.py."""

    def _stack(self, make, nfeat, nhid, nclass, nlayers, with_bn):
        self.layers = nn.ModuleList([])
        if nlayers == 1:
            self.layers.append(make(nfeat, nclass))
        else:
            if with_bn:
                self.bns = nn.ModuleList([nn.BatchNorm1d(nhid)])
            self.layers.append(make(nfeat, nhid))
            for _ in range(nlayers - 2):
                self.layers.append(make(nhid, nhid))
                if with_bn:
                    self.bns.append(nn.BatchNorm1d(nhid))
            self.layers.append(make(nhid, nclass))

    def _setup(self, nfeat, nclass, dropout, lr, weight_decay, with_relu, with_bias, with_bn, device):
        if device is None:
            raise ValueError("Please specify 'device'!")
        self.device = device
        self.nfeat, self.nclass = nfeat, nclass
        self.dropout, self.lr = dropout, lr
        self.weight_decay = weight_decay if with_relu else 0  # a linear model trains without decay
        self.with_relu, self.with_bn, self.with_bias = with_relu, with_bn, with_bias
        self.output = None
        self.multi_label = None

    def _hidden(self, ix, x):
        if ix != len(self.layers) - 1:
            x = self.bns[ix](x) if self.with_bn else x
            if self.with_relu:
                x = F.relu(x)
            x = F.dropout(x, self.dropout, training=self.training)
        return x

    def initialize(self):
        for layer in self.layers:
            layer.reset_parameters()
        if self.with_bn:
            for bn in self.bns:
                bn.reset_parameters()

    def _set_labels(self, labels):
        self.multi_label = len(labels.shape) > 1
        self.loss = torch.nn.BCELoss() if self.multi_label else F.nll_loss
        return labels.float() if self.multi_label else labels

    def _best_val_loop(self, train_out, eval_out, labels_val, val_rows, train_iters, log_every=0):
        """600-epoch style loop: Adam, LR/10 restart at half, eval forward every epoch, weights of
        the first strictly best validation accuracy."""
        optimizer = optim.Adam(self.parameters(), lr=self.lr, weight_decay=self.weight_decay)
        best_acc_val = 0
        weights = deepcopy(self.state_dict())
        for i in range(train_iters):
            if i == train_iters // 2:
                optimizer = optim.Adam(self.parameters(), lr=self.lr * 0.1, weight_decay=self.weight_decay)
            self.train()
            optimizer.zero_grad()
            loss_train = train_out()
            loss_train.backward()
            optimizer.step()
            if log_every and i % log_every == 0:
                print("Epoch {}, training loss: {}".format(i, loss_train.item()))
            with torch.no_grad():
                self.eval()
                output = eval_out()
                sel = output if val_rows is None else output[val_rows]
                acc_val = accuracy(sel, labels_val)
                if acc_val > best_acc_val:
                    best_acc_val = acc_val
                    self.output = output
                    weights = deepcopy(self.state_dict())
        self.load_state_dict(weights)


class GCN(_Trainable):
    """models/gcn.py GCN (GraphConvolution stack, log-softmax head)."""

    def __init__(self, nfeat, nhid, nclass, nlayers=2, dropout=0.5, lr=0.01, weight_decay=5e-4,
                 with_relu=True, with_bias=True, with_bn=False, device=None):
        super().__init__()
        self._setup(nfeat, nclass, dropout, lr, weight_decay, with_relu, with_bias, with_bn, device)
        self._stack(lambda a, b: GraphConvolution(a, b, with_bias=with_bias), nfeat, nhid, nclass,
                    nlayers, with_bn)

    def forward(self, x, adj):
        for ix, layer in enumerate(self.layers):
            x = self._hidden(ix, layer(x, adj))
        return torch.sigmoid(x) if self.multi_label else F.log_softmax(x, dim=1)

    def fit_with_val(self, features, adj, labels, data, train_iters=200, initialize=True,
                     verbose=False, normalize=True, noval=False, full=False, **kwargs):
        """Train on (features, adj, labels) — the distilled graph — scoring data's full graph (or
        its val graph with ``noval``) every epoch (models/gcn.py:249-342)."""
        if initialize:
            self.initialize()
        self.features = _feat(features, self.device)
        adj = adj.to(self.device) if isinstance(adj, torch.Tensor) else adj
        self.adj_norm = normalize_any(adj) if normalize else adj
        labels = labels.to(self.device) if isinstance(labels, torch.Tensor) else torch.LongTensor(labels).to(self.device)
        labels = self._set_labels(labels)
        self.labels = labels
        if noval:
            feat_full, adj_full, val_rows = data.feat_val, data.adj_val, None
        else:
            feat_full, adj_full, val_rows = data.feat_full, data.adj_full, data.idx_val
        feat_full = _feat(feat_full, self.device)
        adj_full_norm = _eval_graph(data, "val" if noval else "full", adj_full, self.device)
        labels_val = torch.LongTensor(data.labels_val).to(self.device)
        if verbose:
            print("=== training gcn model ===")

        def train_out():
            out = self.forward(self.features, self.adj_norm)
            return self.loss(out[data.idx_train], labels) if full else self.loss(out, labels)

        self._best_val_loop(train_out, lambda: self.forward(feat_full, adj_full_norm), labels_val,
                            val_rows, train_iters)

    @torch.no_grad()
    def predict(self, features=None, adj=None):
        """log-probabilities; adj is normalised first (models/gcn.py:362-389)."""
        self.eval()
        if features is None and adj is None:
            return self.forward(self.features, self.adj_norm)
        self.features = _feat(features, self.device)
        self.adj_norm = normalize_any(_as_device_graph(adj, self.device))
        return self.forward(self.features, self.adj_norm)


def _eval_graph(data, role, adj, device):
    """The normalised full (or val) graph of the per-epoch evaluation, built once per data object
    and device (the reference re-normalises it on the host at every fit)."""
    cache = data.__dict__.setdefault("_gdd_norm", {})
    key = (role, str(torch.device(device)))
    g = cache.get(key)
    if g is None:
        g = cache[key] = normalize_any(_as_device_graph(adj, device))
    return g


class MLP(_Trainable):
    """models/gcn.py MLP (nn.Linear stack); ``mode='e'`` also returns the last layer's logits."""

    def __init__(self, nfeat, nhid, nclass, nlayers=2, dropout=0.5, lr=0.01, weight_decay=5e-4,
                 with_relu=True, with_bias=True, with_bn=False, device=None):
        super().__init__()
        self._setup(nfeat, nclass, dropout, lr, weight_decay, with_relu, with_bias, with_bn, device)
        self._stack(nn.Linear, nfeat, nhid, nclass, nlayers, with_bn)

    def forward(self, x, mode="t"):
        for ix, layer in enumerate(self.layers):
            x = self._hidden(ix, layer(x))
        out = torch.sigmoid(x) if self.multi_label else F.log_softmax(x, dim=1)
        return out if mode == "t" else (out, x)

    def fit_with_val(self, features, adj, labels, idx_train, data, train_iters=200, initialize=True,
                     verbose=False, normalize=True, noval=False, **kwargs):
        """models/gcn.py:515-606: train on features[idx_train] (labels are the train labels),
        validate on data.idx_val of the same features. ``adj`` is not used by an MLP (the
        reference normalises it anyway; skipped here, no numerical effect)."""
        if initialize:
            self.initialize()
        self.features = _feat(features, self.device)
        labels = labels.to(self.device) if isinstance(labels, torch.Tensor) else torch.LongTensor(labels).to(self.device)
        labels = self._set_labels(labels)
        self.labels = labels
        labels_val = torch.LongTensor(data.labels_val).to(self.device)
        val_rows = None if noval else data.idx_val
        self._best_val_loop(lambda: self.loss(self.forward(self.features)[idx_train], labels),
                            lambda: self.forward(self.features), labels_val, val_rows, train_iters,
                            log_every=100)

    @torch.no_grad()
    def predict(self, features=None, adj=None, mode="t"):
        self.eval()
        if features is not None:
            self.features = features
        return self.forward(self.features, mode)


class MLP_Induct(MLP):
    """models/gcn.py MLP_Induct (:705-861): the inductive agent's MLP — trained on the train role's
    features and labels, validated on the val role's (its own sub-graph), no per-100-epoch print."""

    def fit_with_val(self, feat_train, labels_train, feat_val, labels_val, train_iters=200,
                     initialize=True, **kwargs):
        if initialize:
            self.initialize()
        feat_train = _feat(feat_train, self.device)
        feat_val = _feat(feat_val, self.device)
        labels_train = self._set_labels(labels_train.to(self.device))
        labels_val = labels_val.to(self.device)
        labels_val = labels_val.float() if self.multi_label else labels_val
        self._best_val_loop(lambda: self.loss(self.forward(feat_train), labels_train),
                            lambda: self.forward(feat_val), labels_val, None, train_iters)

    @torch.no_grad()
    def predict(self, feat_test, mode="t"):
        self.eval()
        return self.forward(feat_test, mode)
