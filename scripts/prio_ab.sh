# Same-box A/B of the step-queue hot-step issue priority (NMPC_SCHED_PRIO=1 default / 0 off):
# three alternating bench runs each (config 3 default workload); lines under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
TAG=${1:-prio}
for rep in 1 2 3; do
  for pr in 1 0; do
    NMPC_SCHED_PRIO=$pr timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline > $O/${TAG}_p${pr}_${rep}.json 2> $O/${TAG}_p${pr}_${rep}.err || exit $?
  done
done
echo prio ab done
