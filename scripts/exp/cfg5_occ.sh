# Dev: config-5 throughput against workgroups per CU (LDS padding caps residency)
set -o pipefail
cd $GRAFT_REPO_ROOT
for lds in 0 40960 53248 65536; do
  NMPC_LDS_BYTES=$lds timeout -k 10 300 python -u bench.py --config 5 --batch 8192 --no-per-step --no-cpu-baseline > gpurun_out/occ5_$lds.json 2> gpurun_out/occ5_$lds.err || exit $?
done
echo done
