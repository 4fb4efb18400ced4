# One GPU pass (run on the box): -m gpu suite, smoke, default bench; logs under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --tb=short --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
echo "all done tests_rc=$rc"
