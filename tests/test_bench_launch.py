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


@pytest.mark.parametrize("n", [2, 3, 8])
def test_bench_gpus_n_spawns_n_ranks(tmp_path, monkeypatch, n):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    line = _line(tmp_path, ["--gpus", str(n), "--timer-steps", "1"] + SMALL)
    assert line["n_gpus"] == n
    assert line["scaling"] == "strong"             # cfg's own graph split n ways
    assert line["steps"] == 2 and line["value"] > 0
    # 2 layers x (engages + rev_engages) of the scaled cfg2 graph (10k engages)
    assert line["config"]["edges_per_step"] == 2 * 2 * 10_000
    assert line["config"]["parallelism"].startswith(f"dst-partitioned x{n}")
    assert line["loss"] == line["loss"] and 0.5 < line["loss"] < 5.0   # global (summed) loss
    assert line["cpu_baseline"] is None             # rank 0 at N=1 only
    # every collective of the sharded step, in issue order, with its wait / stall over ranks
    # (VERDICT r5 #2): the layer-1 all-gather, the layer-2 partial sums' reduce-scatters (two
    # row ranges), the loss's post table as one broadcast per source rank, the backward's
    # reduce-scatter of dP, the slice-gradient all-gathers and the layer-1 post-table gradient's
    # reduce-scatters (two ranges each), the weight all-reduce
    d = line["dist"]
    ops = [c["op"] for c in d["collectives"]]
    assert ops == (["all_gather", "reduce_scatter", "reduce_scatter"]
                   + [f"broadcast[src={q}]" for q in range(n)]
                   + ["reduce_scatter", "all_gather", "all_gather", "reduce_scatter",
                      "reduce_scatter", "all_reduce"])
    assert d["collectives_per_step"] == len(ops) == 9 + n and not d["positions_differ"]
    for c in d["collectives"]:
        assert 0 <= c["stall_ms_min"] <= c["stall_ms_max"] <= c["wait_ms_max"] + 1e-6
        assert c["wait_ms_min"] <= c["wait_ms_max"] and c["MB"] > 0
    assert 0 < d["compute_ms_min"] <= d["compute_ms_max"]
    assert d["stall_ms_max"] >= d["stall_ms_min"] >= 0


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


# ----------------------------------------------------------------------------- measurement tail
def _cfg4_kernels():
    """A per-kernel summary shaped like the cfg4 timer run's (ops.KernelTimer.summary()): 5
    steps; bytes / flops per SURVEY §8d and the K3 byte counts."""
    E, U, P, d = 200_000_000, 9_000_000, 1_000_000, 128

    def rec(launches, ms, nbytes, flops=0, cbytes=None):
        return {"launches": launches, "ms": ms, "bytes": nbytes * launches,
                "cbytes": (cbytes or nbytes) * launches, "flops": flops * launches}
    g = 4 * E * (1 + d) + 4 * (P + 1) + 4 * P * d
    return {
        "gather_fwd[1000000<-9000000]x128": rec(10, 150.2, g, cbytes=4 * U * d),
        "gather_fwd[9000000<-1000000]x128": rec(10, 117.8, 4 * E * (1 + d) + 4 * (U + 1) + 4 * U * d),
        "linear_fwd[9000000x256->128]": rec(5, 15.6, 4 * U * (256 + 128) + 16 * U,
                                            2 * U * 256 * 128),
        "linear_fwd[1000000x256->128]": rec(10, 3.3, 4 * P * (256 + 128), 2 * P * 256 * 128),
        "sort_negatives": rec(5, 14.9, 4 * E * 8),
    }


def test_bench_measurement_tail_runs_on_injected_summaries(monkeypatch):
    """bench.py's N = 1 tail (``_roofline``, ``_one_pass_k1``, ``_projection``, the kernel table)
    on an injected cfg4-shaped kernel summary, on the CPU: no name or key error can first show
    up on the GPU box, and the numbers follow their formulas."""
    kern = _cfg4_kernels()
    cfg = bench.synth.CONFIGS["cfg4"]
    roof = bench._roofline(kern, cfg, 1)
    assert roof["kernel"].endswith("gather_fwd[1000000<-9000000]x128")
    assert roof["algorithmic_bytes_per_launch"] == 4 * 200_000_000 * 129 + 4 * 1_000_001 + 4 * 1_000_000 * 128
    assert abs(roof["avg_launch_us"] - 15020.0) < 1e-6
    assert abs(roof["frac"] - roof["achieved"] / 8000.0) < 1e-3 and 0.8 < roof["frac"] < 0.9

    # _one_pass_k1 end to end with CPU stand-ins for the relation build, the gather and the
    # HIP events (the GPU box runs the real ones)
    import torch
    from truth_recommendation_gnn_amd import graph as G, ops

    class _Ev:
        t = iter([0.0, 17.0])

        def __init__(self, enable_timing=False):
            pass

        def record(self, *a):
            self.ms = next(_Ev.t)

        def elapsed_time(self, other):
            return (other.ms - self.ms) * 3

    calls = []
    monkeypatch.setattr(G, "relation_csr", lambda e, n_src, n_dst: ("csr", n_src, n_dst))
    monkeypatch.setattr(ops, "gather_mean", lambda x, csr: calls.append(
        (ops.GATHER_BLOCK_BYTES, csr)))
    monkeypatch.setattr(torch.cuda, "Event", _Ev)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a: None)
    g = bench.synth.SynthGraph(cfg, {"user": torch.zeros(1, 1), "post": torch.zeros(1, 1)},
                               {bench.synth.ENGAGES: torch.zeros(2, 1, dtype=torch.long)})
    keep = ops.GATHER_BLOCK_BYTES
    one = bench._one_pass_k1(g, cfg, roof)
    assert ops.GATHER_BLOCK_BYTES == keep                     # restored
    assert len(calls) == 4 and all(c[0] == 0 for c in calls)  # unblocked, warm-up + 3 timed
    assert calls[0][1] == ("csr", cfg.num_users, cfg.num_posts)
    assert abs(one["avg_launch_us"] - 17_000.0) < 1e-6
    assert abs(one["frac"] - roof["algorithmic_bytes_per_launch"] / 17e-3 / 8e12) < 1e-4

    proj = bench._projection(kern, "cfg4")
    assert proj["kernel"].endswith("linear_fwd[9000000x256->128]")
    hbm_ms = (4 * 9e6 * 384 + 16 * 9e6) / 8e12 * 1e3
    mfma_ms = 6 * (9e6 / 16) * 8 * 8 * 16 / 1024 / 2.4e9 * 1e3
    assert abs(proj["floor_ms"]["hbm"] - hbm_ms) < 1e-3 and abs(proj["floor_ms"]["mfma"] - mfma_ms) < 1e-3
    # against the launch's own floor ...
    assert proj["bound"] == "hbm" and abs(proj["frac_of_floor"] - hbm_ms / 3.12) < 1e-3
    assert abs(proj["floor_rate"] - 2 * 9e6 * 256 * 128 / (hbm_ms * 1e-3) / 1e12) < 0.1
    # ... and against the chip's bf16 MFMA peak: 6 bf16 products per fp32 product
    tfs = 2 * 9e6 * 256 * 128 / 3.12e-3 / 1e12
    assert abs(proj["achieved"] - tfs) < 0.1 and abs(proj["peak"] - 2500 / 6) < 0.1
    assert abs(proj["frac"] - 6 * tfs / 2500) < 1e-3 and proj["bf16_mfma_frac"] == proj["frac"]
    assert "hbm_frac" not in proj
    # the PMC matrix-pipe busy of the same launch, from the newest committed K3 counter pass
    assert proj["mfma_util"] is not None and 0 < proj["mfma_util"] <= 1
    assert "k_lin_fwd_xs<256, false>" in proj["mfma_util_source"]
    # cfg5's sampled blocks: "[*xK->H]" labels, K = 384 on the split as two column blocks
    n5 = 17_000
    k5 = {"linear_fwd[*x384->128]": {"launches": 4, "ms": 4 * 0.0317,
                                     "bytes": 4 * 4 * n5 * 512, "flops": 4 * 2 * n5 * 384 * 128,
                                     "cbytes": 0}}
    p5 = bench._projection(k5, "cfg5")
    assert p5["method"].startswith("bf16x6") and "two column-block" in p5["method"]
    mfma5 = 6 * (n5 / 16) * 8 * 12 * 16 / 1024 / 2.4e9 * 1e3
    assert abs(p5["floor_ms"]["mfma"] - round(mfma5, 4)) < 1e-9 and 0 < p5["frac_of_floor"] <= 1.0
    assert 0 < p5["frac"] <= 1.0 and p5["mfma_util"] is None    # no counter pass at this shape

    rows = bench._kernel_rows(kern, 5, "cfg4", 1)
    assert rows["gather_fwd[9000000<-1000000]x128"]["cache_assisted"]       # > 8 TB/s
    assert not rows["gather_fwd[1000000<-9000000]x128"]["cache_assisted"]
    for r in rows.values():
        if r["pmc_traffic_over_algorithmic"]:
            assert abs(r["pmc_GB/s"] - r["GB/s"] * r["pmc_traffic_over_algorithmic"]) < 1.0
