# Same-box A/B: alternating bench runs (config 3 unless BENCH_ARGS) of the product and variants,
# optional bitwise dump comparison (AB_DUMP=1); logs under gpurun_out/<tag>_*
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=$1; shift
if [ -n "$AB_DUMP" ]; then
  timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_prod.npz > $O/${TAG}_prod_dump.log 2>&1 || exit $?
  for v in "$@"; do
    NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_$v.npz > $O/${TAG}_${v}_dump.log 2>&1 || exit $?
    python scripts/ab_bitwise.py --compare /tmp/ab_prod.npz /tmp/ab_$v.npz > $O/${TAG}_${v}_cmp.txt 2>&1
  done
fi
for rep in ${AB_REPS:-1 2}; do
  for v in "$@"; do
    NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline ${BENCH_ARGS:-} > $O/${TAG}_${v}_${rep}.json 2> $O/${TAG}_${v}_${rep}.err || exit $?
  done
done
echo ab bench done
