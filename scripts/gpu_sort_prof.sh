cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1; export TMPDIR=/tmp
for cfg in "6 1" "6 0" "9 1"; do set -- $cfg
HGNN_SORT_BITS=$1 HGNN_SORT_LSD=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sortprof_$1_$2 -o run -- python scripts/sort_bench.py --reps 5 > gpurun_out/sortprof.log 2>&1 || exit 1
python - gpurun_out/sortprof_$1_$2/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'hgnn' in r['Name']: print(r['Name'][:60], r['Calls'], r['AverageNs'])
PY
echo ---
done
