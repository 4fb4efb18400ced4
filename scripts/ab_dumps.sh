# Dev: bitwise dumps of variant libraries against the product (config 3), one bench each
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=$1; shift
timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_prod.npz > $O/${TAG}_prod_dump.log 2>&1 || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_$v.npz > $O/${TAG}_${v}_dump.log 2>&1 || exit $?
  python scripts/ab_bitwise.py --compare /tmp/ab_prod.npz /tmp/ab_$v.npz > $O/${TAG}_${v}_cmp.txt 2>&1
done
for v in $BENCH_V; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline > $O/${TAG}_${v}_bench.json 2> $O/${TAG}_${v}_bench.err || exit $?
done
echo dumps done
