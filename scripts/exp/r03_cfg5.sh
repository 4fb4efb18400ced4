set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
T=${1:-r03d}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --tb=short --timeout 600 --timeout-method thread > $O/${T}_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u bench.py --config 5 --batch 8192 --no-per-step --no-cpu-baseline > $O/${T}_cfg5_bench.json 2> $O/${T}_cfg5_bench.err || exit $?
timeout -k 10 300 python -u bench.py --no-per-step --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || exit $?
echo done
