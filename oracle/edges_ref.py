"""CPU restatement of the reference's host edge construction (TEST INFRASTRUCTURE ONLY: imported by
tests/ as the checker of ``truth_recommendation_gnn_amd.edges``; never by the product).

* ``build_edge_index_safe`` follows ``train_gnn.py:40-73``: ``iterrows``, three ``dict.get`` per
  row, a row is kept only if all three ids map; returns ``[engager; post]`` and
  ``[post; target_user]`` as int64 ``[2, M]``.
* ``build_test_edges`` follows ``test_gnn.py:34-55`` (engager and post only).
* ``map_edges`` follows ``build_graph.py:383-402``: ``Series.map(dict)`` on both columns,
  ``dropna()``, ``astype(int)``.

Parity: the restatement is the reference's own loop (dict semantics, row order), so it is pinned by
construction; the reference ships no fixture for it.
"""
from __future__ import annotations

import pandas as pd
import torch


def build_edge_index_safe(df: pd.DataFrame, user_to_idx, post_to_idx):
    engager, post_global, target_user = [], [], []
    for _, row in df.iterrows():
        u_eng = user_to_idx.get(row["engager"])
        u_tgt = user_to_idx.get(row["target_user"])
        p = post_to_idx.get(row["post_id"])
        if u_eng is not None and u_tgt is not None and p is not None:
            engager.append(u_eng)
            post_global.append(p)
            target_user.append(u_tgt)
    e = torch.tensor(engager, dtype=torch.long)
    p = torch.tensor(post_global, dtype=torch.long)
    t = torch.tensor(target_user, dtype=torch.long)
    return torch.stack([e, p], dim=0), torch.stack([p, t], dim=0)


def build_test_edges(df: pd.DataFrame, user_to_idx, post_to_idx):
    engager, post_global = [], []
    for _, row in df.iterrows():
        u = user_to_idx.get(row["engager"])
        p = post_to_idx.get(row["post_id"])
        if u is not None and p is not None:
            engager.append(u)
            post_global.append(p)
    return torch.tensor([engager, post_global], dtype=torch.long).reshape(2, -1)


def map_edges(df: pd.DataFrame, src_col, src_map, dst_col, dst_map):
    m = df[[src_col, dst_col]].copy()
    m[src_col] = m[src_col].map(src_map)
    m[dst_col] = m[dst_col].map(dst_map)
    m = m.dropna().astype("int64")
    return torch.tensor(m[[src_col, dst_col]].values.T, dtype=torch.long).reshape(2, -1)
