cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for L in "" libhgnn_occ16.so libhgnn_occ8.so; do for U in 4 8; do
  HGNN_LIB=$L HGNN_G128_U=$U timeout -k 10 200 python -u scripts/fuse_occupancy_probe.py 2>&1 | grep '^{' || exit 1
done; done
