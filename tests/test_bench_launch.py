"""bench.py's launcher and sharded step on CPU (gloo): ``bench.py --gpus 2`` run without
``torch.distributed.run`` starts two rank processes itself, each runs the destination-partitioned
training step (``UserShard.step`` -> ``sync_grads`` -> Adam) with plain-torch compute ops injected
(``dist_torch_impl.TorchImpl`` — the HIP kernels are covered by the -m gpu tests), and rank 0
prints one JSON line that says ``n_gpus: 2``.  Also: a world size that disagrees with ``--gpus``
is refused, and ``--device cpu`` without injected ops is refused (no CPU product path)."""
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(__file__))
import bench  # noqa: E402
from dist_torch_impl import TorchImpl  # noqa: E402

SMALL = ["--device", "cpu", "--config", "cfg2", "--scale", "0.0005", "--steps", "2",
         "--warmup", "1"]


def _line(tmp_path, argv):
    out = tmp_path / "line.json"
    bench.main(argv + ["--json-out", str(out)], impl_factory=TorchImpl)
    return json.loads(out.read_text())


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_spawns_n_ranks(tmp_path, monkeypatch, n):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    line = _line(tmp_path, ["--gpus", str(n)] + SMALL)
    assert line["n_gpus"] == n
    assert line["scaling"] == "strong"             # cfg's own graph split n ways
    assert line["steps"] == 2 and line["value"] > 0
    # 2 layers x (engages + rev_engages) of the scaled cfg2 graph (10k engages)
    assert line["config"]["edges_per_step"] == 2 * 2 * 10_000
    assert line["config"]["parallelism"].startswith(f"dst-partitioned x{n}")
    assert line["loss"] == line["loss"] and 0.5 < line["loss"] < 5.0   # global (summed) loss
    assert line["cpu_baseline"] is None             # rank 0 at N=1 only


def test_bench_weak_label(tmp_path, monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    line = _line(tmp_path, ["--gpus", "2", "--weak"] + SMALL)
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["edges_per_step"] == 2 * 2 * 2 * 10_000


def test_bench_refuses_world_size_mismatch(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit, match="WORLD_SIZE"):
        bench.main(["--gpus", "8"])


def test_bench_cpu_needs_injected_ops(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    with pytest.raises(SystemExit, match="no CPU product path"):
        bench.main(["--device", "cpu"])


def test_bench_defaults_are_the_north_star_graph():
    a = bench.parse([])
    assert a.config == "cfg4" and a.gpus == 1 and not a.weak
    c = bench.synth.CONFIGS[a.config]
    assert (c.num_users + c.num_posts, c.num_engages, c.dim) == (10_000_000, 200_000_000, 128)
