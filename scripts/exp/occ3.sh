set -o pipefail
cd $GRAFT_REPO_ROOT
for L in 0 53248 81920; do
  NMPC_LDS_BYTES=$L timeout -k 10 300 python -u bench.py --no-per-step --no-cpu-baseline > gpurun_out/occ3_$L.json 2> gpurun_out/occ3_$L.err || exit $?
done
echo done
