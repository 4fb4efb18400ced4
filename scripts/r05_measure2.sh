# round-5 measurement pass 2 (GPU box): phase profiles (diagnostic builds under
# variants/), the bounding chain's trace, raw step times, config-5 bench + rocprofv3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=${1:-r05}
bash scripts/r05_phases.sh $TAG || exit 1
timeout -k 10 120 python -u scripts/chain_trace.py > $O/${TAG}_chain_trace.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/step_times.py $O/${TAG}_steptimes.npz > $O/${TAG}_step_times.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config 5 --batch 8192 --no-per-step > $O/${TAG}_cfg5_bench.json 2> $O/${TAG}_cfg5_bench.err || exit 1
BENCH_ARGS="--config 5 --batch 8192" bash scripts/profile_round.sh ${TAG}_cfg5 || exit 1
echo measure2 done
