# GPU test pass (run on the box): the full -m gpu suite, output under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --tb=short --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
