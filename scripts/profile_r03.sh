# round-3 profiles (GPU box): config 3 (bench default) and config 5 (B = 8192)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/profile_round.sh r03 || exit $?
BENCH_ARGS="--config 5 --batch 8192" bash scripts/profile_round.sh r03_cfg5 || exit $?
echo profiles done
