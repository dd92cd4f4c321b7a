cd $GRAFT_REPO_ROOT
for a in 1 2 8 9; do echo "ABL=$a"; HGNN_SCORE_ABL=$a timeout -k 10 300 python scripts/microbench.py --reps 10 2>&1 | grep "edge_score"; done
SKIP_TESTS=1 PROFILE=r1b bash scripts/gpu_round.sh --steps 20 --warmup 3
