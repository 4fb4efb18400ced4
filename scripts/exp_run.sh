# Dev: A/B measurement of a variant library on the GPU box (bench line, phase profile of
# the stamps build, the longest chain alone, fixture parity); logs under gpurun_out/<tag>_*
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; T=$1; L=$PWD/$2; LS=${3:+$PWD/$3}
NMPC_LIB=$L timeout -k 10 300 python -u bench.py --no-per-step --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || exit $?
if [ -n "$LS" ]; then
  NMPC_LIB=$LS timeout -k 10 200 python -u scripts/phase_profile.py 3 1024 > $O/${T}_phase.log 2>&1 || exit $?
  NMPC_LIB=$LS timeout -k 10 200 python -u scripts/resto_profile.py 1024 > $O/${T}_resto.log 2>&1 || exit $?
fi
NMPC_LIB=$L timeout -k 10 200 python -u scripts/chain_trace.py 2284 > $O/${T}_chain.log 2>&1 || exit $?
if [ -n "$4" ]; then
  NMPC_LIB=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fixtures.py > $O/${T}_fix.log 2>&1
  echo "fixtures rc=$?"
fi
echo exp done
