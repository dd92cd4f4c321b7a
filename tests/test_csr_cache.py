"""The CSR cache (graph._CsrCache) ties an entry's lifetime to its edge tensor's: freed tensors
leave no entry behind, an in-place change replaces the entry, and a live tensor keeps hitting.
The structure built per entry is stubbed here (CPU); the GPU test in test_gpu_parity.py builds
real RelationCSRs and checks the device allocator returns to its baseline."""
import gc

import pytest
import torch

from truth_recommendation_gnn_amd import graph


class _Fake:
    built = 0

    def __init__(self, edge_index, n_src, n_dst, chunk=None):
        type(self).built += 1
        self.n_src, self.n_dst = n_src, n_dst


@pytest.fixture
def cache(monkeypatch):
    monkeypatch.setattr(graph, "RelationCSR", _Fake)
    _Fake.built = 0
    return graph._CsrCache(cap=64)


def test_entries_die_with_their_edge_tensors(cache):
    for i in range(100):        # inference.py:410-419 builds a fresh graph per user
        ei = torch.randint(0, 10, (2, 50 + i))
        cache.get(ei, 10, 10)
        del ei
    gc.collect()
    assert len(cache) == 0
    assert _Fake.built == 100


def test_live_tensor_hits_and_in_place_change_replaces_entry(cache):
    ei = torch.randint(0, 10, (2, 40))
    a = cache.get(ei, 10, 10)
    assert cache.get(ei, 10, 10) is a
    assert len(cache) == 1
    ei[0, 0] = (int(ei[0, 0]) + 1) % 10           # new version: a stale CSR must not be reused
    b = cache.get(ei, 10, 10)
    assert b is not a and len(cache) == 1
    del ei
    gc.collect()
    assert len(cache) == 0


def test_cap_bounds_live_entries(cache):
    cache.cap = 4
    keep = [torch.randint(0, 10, (2, 30)) for _ in range(6)]
    for t in keep:
        cache.get(t, 10, 10)
    assert len(cache) == 4
    first = cache.get(keep[-1], 10, 10)          # most recent: still cached
    assert _Fake.built == 6 and first is not None
    del keep, t
    gc.collect()
    assert len(cache) == 0


def test_view_objects_of_one_storage_get_distinct_entries(cache):
    base = torch.randint(0, 10, (2, 30))
    v1 = base[:, :20]
    cache.get(v1, 10, 10)
    del v1
    gc.collect()
    assert len(cache) == 0                       # the view died, the base lives: entry dropped
