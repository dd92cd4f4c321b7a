"""The cfg5 bench's pipeline (the next batch sampled and staged on a side stream under the running
replay; by default into the live buffers of the second of two recorded steps replayed in turn)
trains exactly the steps the unpipelined loop trains: the same end-of-run loss, bitwise, with
the sync-free LinkSampler (one or two recorded steps) and with the eager sampler.  Rounds 4-5 did not hold this — the
side stream read the epoch's edge permutation (and the batch's edge ids) before the main stream
had written them, so the capture's warm-up trained on a garbled batch 0 (their 0.75 loss after
320 steps against 1.30 unpipelined)."""
import json

import pytest

import bench

pytestmark = pytest.mark.gpu

SMALL = ["--config", "cfg5", "--scale", "0.005", "--batch-seeds", "128", "--steps", "12",
         "--warmup", "3", "--timer-steps", "0", "--no-cpu-baseline"]


def _loss(tmp_path, extra):
    out = tmp_path / "line.json"
    bench.main(SMALL + extra + ["--json-out", str(out)])
    return json.loads(out.read_text())["loss"]


def test_pipelined_cfg5_steps_equal_unpipelined(tmp_path):
    ref = _loss(tmp_path, ["--no-prefetch", "--single-buffer"])
    assert _loss(tmp_path, []) == ref                        # two recorded steps in turn
    assert _loss(tmp_path, ["--single-buffer"]) == ref      # one, with the staging copy
    assert _loss(tmp_path, ["--eager-sampler"]) == ref
