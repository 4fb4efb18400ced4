# round-5 measurement pass 1 (GPU box): the default bench line (with its CPU baseline),
# then the rocprofv3 passes of scripts/profile_round.sh for config 3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=${1:-r05}
timeout -k 10 300 python -u bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit 1
bash scripts/profile_round.sh $TAG || exit 1
echo measure done
