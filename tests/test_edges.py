"""Device edge construction from raw ids (edges.py, csrc/idmap.hip) against the
reference's host loops restated in oracle/edges_ref.py (train_gnn.py:40-73, test_gnn.py:34-55,
build_graph.py:383-402).  Integer work: results must be identical (rows, order, values)."""
import numpy as np
import pandas as pd
import pytest
import torch

from oracle import edges_ref

DEV = torch.device("cuda")


def _frame(seed, n_rows, n_users, n_posts, miss=0.05, id_style="str"):
    """Activity-like frame: engager / target_user user ids, post_id local ids; a fraction of
    every column unmapped (unknown ids, None, NaN, out-of-range posts)."""
    rng = np.random.default_rng(seed)
    if id_style == "str":
        users = [f"u{i}" if i % 7 else f"user_é_{i:06d}_long_suffix" for i in range(n_users)]
        users[0] = ""                                   # empty string is a valid key
    else:
        users = list(rng.permutation(10 * n_users)[:n_users].astype(np.int64) - 3 * n_users)
    user_to_idx = {u: i for i, u in enumerate(sorted(users, key=str))}
    post_to_idx = {i: n_users + i for i in range(n_posts)}

    def col(pool, unknown):
        v = [pool[j] for j in rng.integers(0, len(pool), n_rows)]
        for j in np.flatnonzero(rng.random(n_rows) < miss):
            v[j] = unknown[int(rng.integers(0, len(unknown)))]
        return v

    unk_users = (["nobody", "u", "U1", None, "u1 "] if id_style == "str"
                 else [10 ** 12, -10 ** 12, None])
    df = pd.DataFrame({
        "engager": col(users, unk_users),
        "target_user": col(users, unk_users),
        "post_id": col(list(range(n_posts)), [n_posts + 5, -1, None]),
        "interaction": ["QT"] * n_rows,
    })
    return df, user_to_idx, post_to_idx


# ----------------------------------------------------------------------------- CPU
def test_oracle_known_answer():
    df = pd.DataFrame({"engager": ["a", "b", "zz", "c"], "target_user": ["b", "a", "a", None],
                       "post_id": [0, 1, 2, 0]})
    um, pm = {"a": 0, "b": 1, "c": 2}, {0: 3, 1: 4, 2: 5}
    eng, auth = edges_ref.build_edge_index_safe(df, um, pm)
    assert eng.tolist() == [[0, 1], [3, 4]] and auth.tolist() == [[3, 4], [1, 0]]
    assert edges_ref.build_test_edges(df, um, pm).tolist() == [[0, 1, 2], [3, 4, 3]]
    assert edges_ref.map_edges(df, "engager", um, "post_id", pm).tolist() == [[0, 1, 2],
                                                                              [3, 4, 3]]
    empty = df.iloc[:0]
    assert edges_ref.build_edge_index_safe(empty, um, pm)[0].shape == (2, 0)
    assert edges_ref.build_test_edges(empty, um, pm).shape == (2, 0)


def test_oracle_forms_agree():
    df, um, pm = _frame(3, 500, 60, 40)
    a = edges_ref.build_test_edges(df, um, pm)
    b = edges_ref.map_edges(df, "engager", um, "post_id", pm)
    assert torch.equal(a, b)


def test_query_encoding_follows_python_equality():
    from truth_recommendation_gnn_amd import edges
    q = edges._encode(pd.Series([1.0, 2.5, np.nan, -4.0]))
    assert q.ints[0].tolist()[0] == 1 and q.ints[1].tolist() == [1, 0, 0, 1]
    q = edges._encode(pd.Series(["a", None, "bc"]))
    offs, data, valid = q.strs
    assert offs.tolist() == [0, 1, 1, 3] and bytes(data[:3]) == b"abc" and valid.tolist() == [1, 0, 1]
    q = edges._encode(pd.Series(["7", 7, 7.0, True, None, 2.5], dtype=object))
    assert q.ints[1].tolist() == [0, 1, 1, 1, 0, 0] and q.ints[0][1:4].tolist() == [7, 7, 1]
    assert q.strs[2].tolist() == [1, 0, 0, 0, 0, 0]
    q = edges._encode(pd.Series(["a", None, "bc"], dtype="string[pyarrow]"))
    assert q.strs[0].tolist() == [0, 1, 1, 3] and q.strs[2].tolist() == [1, 0, 1]
    q = edges._encode(np.array([1, 2 ** 63 + 1], dtype=np.uint64))
    assert q.ints[1].tolist() == [1, 0]


def test_idmap_rejects_bad_maps_before_any_device_work():
    from truth_recommendation_gnn_amd import edges
    with pytest.raises(ValueError):
        edges.IdMap({"a": 1}, device="cpu")             # device checked first: no CPU path


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_rows,id_style", [(0, 3000, "str"), (1, 2000, "int"),
                                                  (2, 1, "str"), (4, 40000, "str")])
def test_build_edge_index_safe_matches_reference_loop(seed, n_rows, id_style):
    from truth_recommendation_gnn_amd import edges
    df, um, pm = _frame(seed, n_rows, 300, 200, id_style=id_style)
    ref_e, ref_a = edges_ref.build_edge_index_safe(df, um, pm)
    got_e, got_a = edges.build_edge_index_safe(df, um, pm, device=DEV)
    assert got_e.dtype == torch.int64 and got_e.device.type == "cuda"
    assert torch.equal(got_e.cpu(), ref_e) and torch.equal(got_a.cpu(), ref_a)
    if id_style == "str":                               # Arrow-backed string columns
        dfa = df.astype({"engager": "string[pyarrow]", "target_user": "string[pyarrow]"})
        got_e, got_a = edges.build_edge_index_safe(dfa, um, pm, device=DEV)
        assert torch.equal(got_e.cpu(), ref_e) and torch.equal(got_a.cpu(), ref_a)


@pytest.mark.gpu
def test_test_edges_and_map_edges_match_reference():
    from truth_recommendation_gnn_amd import edges
    df, um, pm = _frame(5, 5000, 400, 300, miss=0.2)
    assert torch.equal(edges.build_test_edges(df, um, pm, device=DEV).cpu(),
                       edges_ref.build_test_edges(df, um, pm))
    social = pd.DataFrame({"follower": df["engager"], "followee": df["target_user"][::-1].values})
    um_d = edges.IdMap(um, DEV)                          # one device map serves both columns
    got = edges.map_edges(social, "follower", um_d, "followee", um_d, device=DEV)
    assert torch.equal(got.cpu(), edges_ref.map_edges(social, "follower", um, "followee", um))


@pytest.mark.gpu
def test_numeric_frames_upcast_by_iterrows():
    """An all-numeric frame makes iterrows yield floats; dict.get(3.0) still finds key 3."""
    from truth_recommendation_gnn_amd import edges
    rng = np.random.default_rng(9)
    df = pd.DataFrame({"engager": rng.integers(0, 50, 800), "target_user": rng.integers(0, 50, 800),
                       "post_id": rng.integers(0, 30, 800), "w": rng.random(800)})
    um = {i: i for i in range(0, 50, 2)}
    pm = {i: 100 + i for i in range(30)}
    ref = edges_ref.build_edge_index_safe(df, um, pm)
    got = edges.build_edge_index_safe(df, um, pm, device=DEV)
    assert all(torch.equal(g.cpu(), r) for g, r in zip(got, ref))


@pytest.mark.gpu
def test_mixed_key_types():
    from truth_recommendation_gnn_amd import edges
    m = {"7": 0, 7: 1, "a": 2, 8: 3, True: 4}          # True == 1 in Python
    col = pd.Series(["7", 7, 7.0, "a", 8.0, 1, "8", None, 2.5, "b", np.int64(8)], dtype=object)
    got = edges.IdMap(m, DEV).lookup(col).cpu().tolist()
    assert got == [m.get(v, -1) if v is not None else -1 for v in col.tolist()]


@pytest.mark.gpu
def test_idmap_at_scale_matches_dict_get():
    """1M string keys (with shared prefixes), 4M queries of which 1/4 are absent."""
    from truth_recommendation_gnn_amd import edges
    rng = np.random.default_rng(11)
    n = 1 << 20
    keys = [f"user_{i:08x}" + ("x" * int(i % 23)) for i in rng.permutation(n)]
    m = {k: i * 3 for i, k in enumerate(keys)}
    pick = rng.integers(0, n, 4 * n)
    q = np.array(keys, dtype=object)[pick]
    absent = rng.random(4 * n) < 0.25
    q[absent] = [s + "?" for s in q[absent]]
    ref = pd.Series(q).map(m).fillna(-1).astype(np.int64).to_numpy()
    got = edges.IdMap(m, DEV).lookup(pd.Series(q)).cpu().numpy()
    assert np.array_equal(got, ref)


@pytest.mark.gpu
def test_edge_cases():
    from truth_recommendation_gnn_amd import edges
    df, um, pm = _frame(6, 100, 20, 10)
    e, a = edges.build_edge_index_safe(df.iloc[:0], um, pm, device=DEV)
    assert e.shape == (2, 0) and a.shape == (2, 0)
    e, a = edges.build_edge_index_safe(df, {}, pm, device=DEV)      # nothing maps
    assert e.shape == (2, 0)
    t = edges.IdMap(pm, DEV).lookup(torch.tensor([0, 9, 10, -1], device=DEV))
    assert t.tolist() == [20, 29, -1, -1]
    with pytest.raises(ValueError):
        edges.IdMap({"a": -1}, DEV)
    with pytest.raises(TypeError):
        edges.IdMap({("a", 1): 0}, DEV)


@pytest.mark.gpu
def test_string_lengths_and_alignments():
    """Word-wide loads: every length 0..40 at every byte alignment, prefixes of each other, and
    the last string of the buffer (the kernels read into the 16-B tail padding)."""
    from truth_recommendation_gnn_amd import edges
    keys = ["x" * n for n in range(0, 41, 2)] + ["ab" * n + "c" for n in range(12)]
    m = {k: i for i, k in enumerate(keys)}
    queries = []
    for pad in range(4):                       # shifts every following string's alignment
        queries += ["p" * pad] + ["x" * n for n in range(41)] + ["ab" * n for n in range(12)]
        queries += ["ab" * n + "c" for n in range(12)] + ["ab" * n + "d" for n in range(12)]
    queries.append(keys[-1])                   # ends the buffer
    got = edges.IdMap(m, DEV).lookup(pd.Series(queries)).cpu().tolist()
    assert got == [m.get(q, -1) for q in queries]
