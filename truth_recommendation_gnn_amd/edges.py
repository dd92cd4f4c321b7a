"""Edge lists from raw entity ids, built on the device (the step before the path).

The reference maps entity ids to node indices on the host, one DataFrame row at a time:

* ``build_edge_index_safe(df, user_to_idx, post_to_idx)`` (``train_gnn.py:40-73``): per row three
  ``dict.get`` calls; rows with any unmapped id are skipped; returns the engagement edges
  ``[engager, post]`` and the authorship edges ``[post, target_user]``;
* ``build_test_edges(df, user_to_idx, post_to_idx)`` (``test_gnn.py:34-55``): the same for
  ``[engager, post]`` only;
* ``Series.map(dict)`` + ``dropna()`` for the social / engage / author lists of
  ``build_graph.py:383-402`` (``map_edges`` here).

Here each dictionary becomes an ``IdMap``, an open-addressing table in HBM (``csrc/idmap.hip``);
the columns are looked up on the GPU and the surviving rows compacted in order by
``hgnn_compact_rows``.  Results equal the reference's (same rows, same order, int64), but live on
the device.  Key and query ids are compared exactly (strings byte for byte after a hash match),
with Python's equality: ``"5" != 5``, ``5.0 == 5``, ``True == 1``; NaN/None never match.

Host work left: converting object string columns to the Arrow layout (offsets + UTF-8 bytes,
pyarrow, ≈150 ns per Python string under the GIL — the floor for Python ``str`` objects; columns
already Arrow-backed, ``dtype="string[pyarrow]"``, go to the device without per-row work) and the
one host sync that sizes the output.
"""
from __future__ import annotations

import numbers
import warnings
from typing import Mapping, Optional, Sequence, Tuple, Union

import numpy as np
import pandas as pd
import pyarrow as pa
import torch

from . import _native as N

_I63 = 2.0 ** 63


def _device(device) -> torch.device:
    dev = torch.device(device)
    if dev.type != "cuda":
        raise ValueError("edge construction runs only on a ROCm GPU (MI355X / gfx950); got "
                         f"device {dev}")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def _arrow_strings(values) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(int64 offsets[n+1], uint8 bytes, uint8 valid[n]) of a string column (None/NaN -> invalid)."""
    if isinstance(values, (pa.Array, pa.ChunkedArray)):
        arr = values.combine_chunks() if isinstance(values, pa.ChunkedArray) else values
        if arr.type != pa.large_string():
            arr = arr.cast(pa.large_string())
    else:
        arr = pa.array(values, type=pa.large_string(), from_pandas=True)
    n = len(arr)
    bufs = arr.buffers()
    offs = np.frombuffer(bufs[1], dtype=np.int64)[arr.offset: arr.offset + n + 1]
    data = (np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None and bufs[2].size
            else np.zeros(0, dtype=np.uint8))
    valid = (~arr.is_null().to_numpy(zero_copy_only=False)).astype(np.uint8)
    return offs, data, valid


def _h2d(a: np.ndarray, dev: torch.device) -> torch.Tensor:
    """Host array -> device tensor.  Arrow-backed arrays are read-only views; they are only read
    here, so torch's non-writable warning does not apply."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def bytes_to_device(data: np.ndarray, dev: torch.device) -> torch.Tensor:
    """A string byte buffer on the device with the 16 B of tail padding the kernels read into."""
    out = torch.zeros(data.size + 16, dtype=torch.uint8, device=dev)
    if data.size:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", UserWarning)
            out[:data.size].copy_(torch.from_numpy(data))
    return out


def _int_like(v) -> Optional[int]:
    """The integer a dict key equal to ``v`` would have, or None (Python equality)."""
    if isinstance(v, (bool, np.bool_)):
        return int(v)
    if isinstance(v, numbers.Integral):
        return int(v)
    if isinstance(v, numbers.Real):
        f = float(v)
        if np.isfinite(f) and f == np.floor(f) and -_I63 <= f < _I63:
            return int(f)
    return None


def _arrow_string_dtype(dt) -> bool:
    if isinstance(dt, pd.StringDtype):
        return dt.storage in ("pyarrow", "pyarrow_numpy")
    if isinstance(dt, pd.ArrowDtype):
        return pa.types.is_string(dt.pyarrow_dtype) or pa.types.is_large_string(dt.pyarrow_dtype)
    return False


class _Queries:
    """One query column split by kind: integer queries and string queries, each full length with
    a validity mask (an element is valid in at most one of the two)."""

    def __init__(self, n: int):
        self.n = n
        self.ints: Optional[Tuple[np.ndarray, np.ndarray]] = None
        self.strs: Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]] = None
        self.ints_dev: Optional[torch.Tensor] = None


def _encode(values) -> _Queries:
    if isinstance(values, torch.Tensor):
        if values.dtype.is_floating_point or values.dtype.is_complex:
            values = values.cpu().numpy()
        else:
            q = _Queries(int(values.numel()))
            q.ints_dev = values.reshape(-1).to(torch.int64)
            return q
    if isinstance(values, (pd.Series, pd.Index)) and _arrow_string_dtype(values.dtype):
        q = _Queries(len(values))                      # Arrow-backed column: no per-row work
        q.strs = _arrow_strings(pa.array(values.array))
        return q
    if isinstance(values, (pd.Series, pd.Index)):
        arr = values.to_numpy()
    else:
        arr = np.asarray(values) if not isinstance(values, list) else np.array(values,
                                                                               dtype=object)
    q = _Queries(len(arr))
    if q.n == 0:
        return q
    kind = arr.dtype.kind
    if kind in "iub":
        a = arr.astype(np.int64, copy=False) if kind != "u" else arr
        if kind == "u":
            valid = (arr < np.uint64(2 ** 63)).astype(np.uint8)
            a = np.where(valid.astype(bool), arr, 0).astype(np.int64)
            q.ints = (a, valid)
        else:
            q.ints = (np.ascontiguousarray(a), np.ones(q.n, dtype=np.uint8))
        return q
    if kind == "f":
        f = arr.astype(np.float64, copy=False)
        with np.errstate(invalid="ignore"):
            valid = np.isfinite(f) & (f == np.floor(f)) & (f >= -_I63) & (f < _I63)
        q.ints = (np.where(valid, f, 0).astype(np.int64), valid.astype(np.uint8))
        return q
    inferred = pd.api.types.infer_dtype(arr, skipna=True)
    if inferred == "string":
        q.strs = _arrow_strings(arr)
        return q
    if inferred == "empty":
        return q
    if inferred in ("integer", "boolean"):
        try:
            q.ints = (arr.astype(np.int64), np.ones(q.n, dtype=np.uint8))
            return q
        except (TypeError, ValueError, OverflowError):
            pass                                # None among the ints, or out of int64 range
    # mixed / numeric objects: classify element by element (slow path, exact semantics)
    iv = np.zeros(q.n, dtype=np.int64)
    ivalid = np.zeros(q.n, dtype=np.uint8)
    svals = [None] * q.n
    for i, v in enumerate(arr):
        if isinstance(v, str):
            svals[i] = v
            continue
        k = _int_like(v)
        if k is not None:
            iv[i], ivalid[i] = k, 1
    if ivalid.any():
        q.ints = (iv, ivalid)
    if any(s is not None for s in svals):
        q.strs = _arrow_strings(svals)
    return q


class IdMap:
    """``dict {entity id: node index}`` as a device hash table (``hgnn_idmap_build``).

    Keys may be strings and/or integers (integral floats count as integers, as in a Python dict);
    values must be integers >= 0.  Build once and reuse for every column that maps through it.
    """

    def __init__(self, mapping: Mapping, device="cuda"):
        self.device = _device(device)
        lib = N.lib()
        keys = list(mapping.keys())
        v64 = np.array(list(mapping.values()))
        if not (v64.dtype.kind in "iu" and (v64.size == 0 or v64.min() >= 0)) or v64.size == 0:
            conv = [_int_like(v) for v in mapping.values()]
            bad = next((kv for kv, c in zip(mapping.items(), conv) if c is None or c < 0), None)
            if bad is not None:
                raise ValueError(f"id map values must be integers >= 0, got {bad[1]!r} for key "
                                 f"{bad[0]!r}")
            v64 = np.array(conv, dtype=np.int64)
        v64 = v64.astype(np.int64)
        kinds = pd.api.types.infer_dtype(keys, skipna=False) if keys else "empty"
        if kinds == "string":
            skeys, svals, ikeys, ivals = keys, v64, [], v64[:0]
        elif kinds in ("integer", "boolean"):
            skeys, svals, ikeys, ivals = [], v64[:0], [int(k) for k in keys], v64
        else:                                   # mixed keys: split element by element
            sidx, iidx, ikeys = [], [], []
            for j, k in enumerate(keys):
                if isinstance(k, str):
                    sidx.append(j)
                    continue
                ki = _int_like(k)
                if ki is None:
                    raise TypeError(f"id map keys must be str or int, got {type(k).__name__} "
                                    f"({k!r})")
                iidx.append(j)
                ikeys.append(ki)
            skeys = [keys[j] for j in sidx]
            svals, ivals = v64[sidx], v64[iidx]
        self.n_keys = len(skeys) + len(ikeys)
        self._int = self._str = None
        dev = self.device
        if ikeys:
            keys = torch.tensor(ikeys, dtype=torch.int64, device=dev)
            self._int = self._table(lib, keys, None, None, len(ikeys),
                                    _h2d(ivals, dev))
        if skeys:
            offs, data, _ = _arrow_strings(skeys)
            offs_d = _h2d(offs, dev)
            data_d = bytes_to_device(data, dev)
            self._str = self._table(lib, None, offs_d, data_d, len(skeys),
                                    _h2d(svals, dev))

    def _table(self, lib, ints, offs, data, n, vals):
        cap = int(lib.hgnn_idmap_capacity(n))
        slots = torch.empty(cap * 16, dtype=torch.uint8, device=self.device)
        N.check(lib.hgnn_idmap_build(N.ptr(ints), N.ptr(offs), N.ptr(data), n, N.ptr(slots), cap,
                                     N.stream_ptr(self.device)), "hgnn_idmap_build")
        return {"cap": cap, "slots": slots, "ints": ints, "offs": offs, "data": data,
                "vals": vals}

    def _lookup(self, t, q_ints, q_offs, q_bytes, q_valid, n, out):
        N.check(N.lib().hgnn_idmap_lookup(
            N.ptr(t["slots"]), t["cap"], N.ptr(t["ints"]), N.ptr(t["offs"]), N.ptr(t["data"]),
            N.ptr(t["vals"]), N.ptr(q_ints), N.ptr(q_offs), N.ptr(q_bytes), N.ptr(q_valid), n,
            N.ptr(out), N.stream_ptr(self.device)), "hgnn_idmap_lookup")

    def lookup(self, values) -> torch.Tensor:
        """``[mapping.get(v, -1) for v in values]`` as a device int64 tensor."""
        q = values if isinstance(values, _Queries) else _encode(values)
        dev = self.device
        out = torch.full((q.n,), -1, dtype=torch.int64, device=dev)
        if q.n == 0:
            return out
        if q.ints_dev is not None:
            if self._int is not None:
                self._lookup(self._int, q.ints_dev.to(dev).contiguous(), None, None, None, q.n,
                             out)
            return out
        if q.ints is not None and self._int is not None:
            iv, ivalid = (_h2d(a, dev) for a in q.ints)
            self._lookup(self._int, iv, None, None, ivalid, q.n, out)
        if q.strs is not None and self._str is not None:
            offs, data, valid = q.strs
            res = out if q.ints is None or self._int is None else torch.empty_like(out)
            self._lookup(self._str, None, _h2d(offs, dev),
                         bytes_to_device(data, dev),
                         _h2d(valid, dev), q.n, res)
            if res is not out:
                torch.maximum(out, res, out=out)   # each element is valid in one kind at most
        return out

    def __len__(self):
        return self.n_keys


MapLike = Union[IdMap, Mapping]


def as_idmap(m: MapLike, device="cuda") -> IdMap:
    return m if isinstance(m, IdMap) else IdMap(m, device)


def compact_rows(cols: Sequence[torch.Tensor], outputs: Sequence[Sequence[int]]):
    """Keep the rows where every column is >= 0, in order.  ``outputs`` lists, per result, the
    columns stacked into it; returns one int64 ``[len(cols_o), kept]`` tensor per result."""
    dev = N.require_device(*cols)
    n = int(cols[0].numel())
    if any(int(c.numel()) != n for c in cols):
        raise ValueError("columns differ in length")
    cols = [c.to(torch.int64).contiguous() for c in cols]
    lib = N.lib()
    ws = N.workspace(lib.hgnn_compact_rows_ws_bytes(n), dev)
    count = torch.empty(1, dtype=torch.int32, device=dev)
    col_arr = N.ptr_array(cols)

    def run(outs, out_col):
        N.check(lib.hgnn_compact_rows(col_arr, len(cols), n, N.ptr_array(outs),
                                      N.int_array(out_col), len(outs), N.ptr(count), N.ptr(ws),
                                      ws.numel(), N.stream_ptr(dev)), "hgnn_compact_rows")

    run([], [])
    m = int(count.item())                      # the one host sync: sizes the outputs
    results, outs, out_col = [], [], []
    for spec in outputs:
        r = torch.empty(len(spec), m, dtype=torch.int64, device=dev)
        results.append(r)
        for j, c in enumerate(spec):
            outs.append(r[j])
            out_col.append(c)
    if m and outs:
        run(outs, out_col)
    return results


def build_edge_index_safe(df, user_to_idx: MapLike, post_to_idx: MapLike, device="cuda"):
    """``train_gnn.py:40-73`` on the device: ``(engage_edge [2,M] = [engager; post],
    author_edge [2,M] = [post; target_user])``, rows with any unmapped id skipped, order kept."""
    dev = _device(device)
    um, pm = as_idmap(user_to_idx, dev), as_idmap(post_to_idx, dev)
    eng = um.lookup(df["engager"])
    post = pm.lookup(df["post_id"])
    tgt = um.lookup(df["target_user"])
    engage, author = compact_rows([eng, post, tgt], [(0, 1), (1, 2)])
    return engage, author


def build_test_edges(df, user_to_idx: MapLike, post_to_idx: MapLike, device="cuda"):
    """``test_gnn.py:34-55`` on the device: ``[2,M] = [engager; post]`` of the mapped rows."""
    dev = _device(device)
    um, pm = as_idmap(user_to_idx, dev), as_idmap(post_to_idx, dev)
    return compact_rows([um.lookup(df["engager"]), pm.lookup(df["post_id"])],
                        [(0, 1)])[0]


def map_edges(df, src_col: str, src_map: MapLike, dst_col: str, dst_map: MapLike,
              device="cuda"):
    """``df[[src, dst]].map(...)`` + ``dropna()`` → ``[2,M]`` (``build_graph.py:383-402``)."""
    dev = _device(device)
    sm = as_idmap(src_map, dev)
    dm = sm if dst_map is src_map else as_idmap(dst_map, dev)
    return compact_rows([sm.lookup(df[src_col]), dm.lookup(df[dst_col])],
                        [(0, 1)])[0]
