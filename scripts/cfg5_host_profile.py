#!/usr/bin/env python3
"""Host-side profile (cProfile) of the cfg5 mini-batch step (bench.py --config cfg5): where the
Python time of a step goes when the GPU is idle between launches."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

args = ["--config", "cfg5", "--steps", "40", "--warmup", "5", "--no-cpu-baseline",
        "--timer-steps", "0"]
pr = cProfile.Profile()
pr.enable()
bench.main(args)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
