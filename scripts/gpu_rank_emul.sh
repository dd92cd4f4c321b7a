#!/bin/bash
# Per-rank compute of the N-GPU weak-scaled bench (scripts/rank_emulation.py) for N = 1, 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
for w in 1 8; do timeout -k 10 200 python scripts/rank_emulation.py --world $w > gpurun_out/rank_emul_$w.json 2>&1 || exit 1; tail -1 gpurun_out/rank_emul_$w.json | cut -c1-80; done
