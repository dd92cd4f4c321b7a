#!/usr/bin/env python3
"""Host-side (Python) profile of the cfg5 mini-batch bench: cProfile over bench.py's cfg5 run
(graph replay steps with the next batch sampled on the side stream), top functions by own time
and cumulative time.  usage: python scripts/cfg5_host_profile.py [steps]"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

steps = sys.argv[1] if len(sys.argv) > 1 else "300"
pr = cProfile.Profile()
pr.enable()
bench.main(["--config", "cfg5", "--steps", steps, "--warmup", "20", "--no-cpu-baseline",
            "--timer-steps", "0"])
pr.disable()
for key in ("tottime", "cumulative"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(40)
    print(s.getvalue())
