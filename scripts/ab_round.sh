# Same-box A/B of variant libraries against the in-tree product: bitwise dumps
# (scripts/ab_bitwise.py: cold batched solve + 20-step fused closed loop, config 3) and
# alternating bench runs (3 each); usage: [BENCH_ARGS="--config 5 --batch 8192" AB_CONFIG=5]
# scripts/ab_round.sh <tag> <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
TAG=$1; shift
timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_prod.npz > $O/${TAG}_prod_dump.log 2>&1 || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_$v.npz > $O/${TAG}_${v}_dump.log 2>&1 || exit $?
  python scripts/ab_bitwise.py --compare /tmp/ab_prod.npz /tmp/ab_$v.npz > $O/${TAG}_${v}_cmp.txt 2>&1
done
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline ${BENCH_ARGS:-} > $O/${TAG}_prod_${rep}.json 2> $O/${TAG}_prod_${rep}.err || exit $?
  for v in "$@"; do
    NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline ${BENCH_ARGS:-} > $O/${TAG}_${v}_${rep}.json 2> $O/${TAG}_${v}_${rep}.err || exit $?
  done
done
echo ab round done
