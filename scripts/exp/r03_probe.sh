# round-3 probe (GPU box): re-run the changed tests, phase profiles (stamps build), the
# longest chain's trace, and the config-5 bench under rocprofv3; logs under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 700 python -u -m pytest -v -s --tb=short --timeout 600 --timeout-method thread tests/test_gpu_reference_runs.py tests/test_gpu_dist.py "tests/test_gpu.py::test_closed_loop_dispatch_order_does_not_change_results" "tests/test_gpu.py::test_closed_loop_check_on_a_side_stream" > $O/r03b_tests.log 2>&1
echo "tests rc=$?"
NMPC_LIB=$PWD/mpc-implementation_amd/nmpc_amd/libnmpc_amd_stamps.so timeout -k 10 200 python -u scripts/phase_profile.py 3 1024 > $O/r03b_phase.log 2>&1 || exit $?
NMPC_LIB=$PWD/mpc-implementation_amd/nmpc_amd/libnmpc_amd_stamps.so timeout -k 10 200 python -u scripts/resto_profile.py 1024 > $O/r03b_resto.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/chain_trace.py 2284 > $O/r03b_chain.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config 5 --batch 8192 --no-per-step --no-cpu-baseline > $O/r03b_cfg5_bench.json 2> $O/r03b_cfg5_bench.err || exit $?
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r03_cfg5_stats -o run -- python3 $R/bench.py --config 5 --batch 8192 --no-per-step --no-cpu-baseline > $R/$O/prof_r03_cfg5_stats.log 2>&1 || exit $?
echo "probe done"
