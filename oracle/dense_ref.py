"""Independent float64 dense-adjacency formulation — TEST INFRASTRUCTURE ONLY.

Pins ``oracle/sage_ref.py`` (itself "parity unpinned" against the reference, see its header):
``SAGEConv`` mean aggregation written as ``D^-1 A X_src W_l^T + b + X_dst W_r^T`` with ``A`` the
dense count matrix (``A[i,j]`` = number of edges j->i, so duplicates count with multiplicity,
self loops are ordinary edges) and ``D = diag(max(rowsum A, 1))`` — a zero-in-degree row gives 0.
Usable only on small graphs (dense [N_dst, N_src]).
"""
from __future__ import annotations

import numpy as np


def adjacency(edge_index: np.ndarray, n_src: int, n_dst: int) -> np.ndarray:
    a = np.zeros((n_dst, n_src), dtype=np.float64)
    if edge_index.shape[1]:
        np.add.at(a, (edge_index[1], edge_index[0]), 1.0)
    return a


def sage_conv_dense(x_src, x_dst, edge_index, w_l, b_l, w_r) -> np.ndarray:
    x_src = np.asarray(x_src, np.float64)
    x_dst = np.asarray(x_dst, np.float64)
    a = adjacency(np.asarray(edge_index), x_src.shape[0], x_dst.shape[0])
    deg = a.sum(1, keepdims=True)
    aggr = (a @ x_src) / np.maximum(deg, 1.0)
    out = aggr @ np.asarray(w_l, np.float64).T + x_dst @ np.asarray(w_r, np.float64).T
    if b_l is not None:
        out = out + np.asarray(b_l, np.float64)
    return out


def softplus(z):
    return np.maximum(z, 0) + np.log1p(np.exp(-np.abs(z)))


def link_loss_dense(user_emb, post_emb, pos_edges, neg_p, pos_weights) -> float:
    u = np.asarray(user_emb, np.float64)
    p = np.asarray(post_emb, np.float64)
    pu, pp = np.asarray(pos_edges[0]), np.asarray(pos_edges[1])
    s_pos = (u[pu] * p[pp]).sum(1)
    s_neg = (u[pu] * p[np.asarray(neg_p)]).sum(1)
    pos_loss = softplus(-s_pos).mean()          # BCEWithLogits(x, 1), mean reduction
    neg_loss = softplus(s_neg).mean()           # BCEWithLogits(x, 0)
    return float(np.asarray(pos_weights, np.float64).mean() * pos_loss + neg_loss)
