# Dev: same-box A/B of variant libraries on config 5 (bench line) and config 3 (bench +
# work-bound batch), then config-5 parity tests on the last variant; logs under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
last=""
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u bench.py --config 5 --batch 8192 --no-per-step --no-cpu-baseline > gpurun_out/c5_${v}.json 2> gpurun_out/c5_${v}.err || exit $?
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u bench.py --no-per-step --no-cpu-baseline > gpurun_out/c3_${v}.json 2> gpurun_out/c3_${v}.err || exit $?
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u bench.py --no-per-step --no-cpu-baseline --batch 16384 > gpurun_out/c3b_${v}.json 2> gpurun_out/c3b_${v}.err || exit $?
  last=$v
done
NMPC_LIB=$PWD/variants/$last.so timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_fixtures.py tests/test_gpu_fp32.py -k "config5 or fp32" > gpurun_out/c5_tests.log 2>&1
echo "tests rc=$?"
