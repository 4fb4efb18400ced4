# round-6 final measurement, in two gpurun calls (each under the 20-minute call limit):
#   part a: -m gpu suite, smoke, the default bench line, the config-3 rocprofv3 passes
#   part b: the config-5 rocprofv3 passes, the step-time diagnostic, the phase builds' profiles
#   part c5: the config-5 rocprofv3 passes alone
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=${2:-r06}
if [ "$1" == "a" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --tb=short --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit $?
  timeout -k 10 400 python -u bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit $?
  echo bench done
  bash scripts/profile_round.sh $TAG || exit 1
  echo "part a done tests_rc=$rc"
elif [ "$1" == "c5" ]; then
  BENCH_ARGS="--config 5 --batch 8192" bash scripts/profile_round.sh ${TAG}_cfg5 || exit 1
  echo "part c5 done"
else
  BENCH_ARGS="--config 5 --batch 8192" bash scripts/profile_round.sh ${TAG}_cfg5 || exit 1
  timeout -k 10 200 python -u scripts/step_times.py $O/${TAG}_step_times.npz > $O/${TAG}_step_times.txt 2>&1 || exit 1
  bash scripts/r06_phases.sh ${TAG}p || exit 1
  echo "part b done"
fi
