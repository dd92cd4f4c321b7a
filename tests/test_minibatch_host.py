"""minibatch.py's staging arena on the CPU: aligned, disjoint views; commit copies the stage to
the live buffers only when something was prepared since the last commit (the capacities are
covered by test_minibatch_caps.py)."""
import torch

from truth_recommendation_gnn_amd import minibatch


def test_arena_views_are_aligned_disjoint_and_committed():
    specs = {"a": (5, torch.int32), "b": (0, torch.int32), "c": (3, torch.float32),
             "d": (70, torch.int32)}
    ar = minibatch._Arena(specs, torch.device("cpu"))
    offs = sorted((o, nb) for o, n, dt, nb in ar.layout.values())
    for (o1, nb1), (o2, _) in zip(offs, offs[1:]):
        assert o1 % 256 == 0 and o1 + nb1 <= o2
    for k, (n, dt) in specs.items():
        assert ar.live[k].numel() == n and ar.live[k].dtype == dt
        assert ar.stage[k].numel() == n and ar.live[k].data_ptr() != ar.stage[k].data_ptr() or n == 0
    ar.wait_committed()                       # a writer marks the stage dirty
    ar.stage["a"].copy_(torch.arange(5, dtype=torch.int32))
    ar.stage["c"].fill_(1.5)
    assert int(ar.live["a"].sum()) == 0
    ar.commit()
    assert ar.live["a"].tolist() == [0, 1, 2, 3, 4] and ar.live["c"].tolist() == [1.5] * 3
    ar.stage["a"].fill_(9)                    # not prepared through wait_committed: no copy
    ar.commit()
    assert ar.live["a"].tolist() == [0, 1, 2, 3, 4]

