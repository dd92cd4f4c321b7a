"""Static block capacities of the captured mini-batch step (minibatch.capacities; CPU)."""
import pytest

from truth_recommendation_gnn_amd import minibatch, synth


def test_capacities_bound_every_level_and_hop():
    rels = [synth.REV_ENGAGES, synth.ENGAGES, synth.SOCIAL, synth.POST_POST]
    cap, ecap = minibatch.capacities(rels, {"user": 1024, "post": 1024}, [15, 10], slack=1024)
    # level 1: the seeds + 15 sampled sources per seed per relation out of each type
    assert cap[0] == {"user": 2048, "post": 2048}
    assert cap[1] == {"user": 1024 + 2 * 15 * 1024 + 1024, "post": 1024 + 2 * 15 * 1024 + 1024}
    assert cap[2]["user"] == 31744 + 2 * 10 * 31744 + 1024
    assert ecap[0] == {et: 15 * 1024 for et in rels}
    assert ecap[1] == {et: 10 * 31744 for et in rels}
    # a type reached only as a source joins the next level
    cap, ecap = minibatch.capacities([("a", "r", "b")], {"b": 10}, [3, 2], slack=4)
    assert cap[1] == {"b": 14, "a": 34} and ecap[0] == {("a", "r", "b"): 30}
    assert ecap[1] == {("a", "r", "b"): 20} and cap[2] == {"b": 14, "a": 30 + 20 + 4}
    with pytest.raises(ValueError, match="bounded fanouts"):
        minibatch.capacities(rels, {"user": 8}, [-1, 3])
