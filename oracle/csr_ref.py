"""numpy COO -> CSR restatement — TEST INFRASTRUCTURE ONLY (bit-exact checker for K5).

The reference never builds a CSR: PyG scatters over the unsorted COO in edge order
(``train_gnn.py:28,55`` keep edges chronological).  The build's CSR is therefore defined as the
*stable* grouping of the COO by the key row: ``perm = argsort(key, kind='stable')``,
``col = other[perm]``, ``rowptr = [0, cumsum(bincount(key, minlength=n_keys))]``.  Stability makes
each row's edge order the reference's edge order, so the HIP result is compared bit for bit.
"""
from __future__ import annotations

import numpy as np


def coo_to_csr(key: np.ndarray, other: np.ndarray, n_keys: int):
    key = np.asarray(key, dtype=np.int64)
    other = np.asarray(other, dtype=np.int64)
    perm = np.argsort(key, kind="stable")
    counts = np.bincount(key, minlength=n_keys) if key.size else np.zeros(n_keys, np.int64)
    rowptr = np.zeros(n_keys + 1, dtype=np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return rowptr.astype(np.int32), other[perm].astype(np.int32), perm.astype(np.int32)


def heavy_plan(rowptr: np.ndarray, chunk: int):
    """Rows with more than ``chunk`` edges and their chunk slots (mirrors graph.py's plan)."""
    deg = np.diff(rowptr.astype(np.int64))
    heavy = np.nonzero(deg > chunk)[0]
    nch = (deg[heavy] + chunk - 1) // chunk
    first = np.zeros(heavy.size + 1, np.int64)
    np.cumsum(nch, out=first[1:])
    return heavy.astype(np.int32), first.astype(np.int32)
