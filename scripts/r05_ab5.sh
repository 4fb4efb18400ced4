# round-5 config-5 A/B (N = 50, moving obstacles, B = 8,192): bitwise dump (1,024 x 5)
# and alternating bench runs of the product and variants/<v>.so
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=$1; shift
AB_CONFIG=5 AB_B=1024 AB_K=5 timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/c5_prod.npz > $O/${TAG}_prod_dump5.log 2>&1 || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so AB_CONFIG=5 AB_B=1024 AB_K=5 timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/c5_$v.npz > $O/${TAG}_${v}_dump5.log 2>&1 || exit $?
  python scripts/ab_bitwise.py --compare /tmp/c5_prod.npz /tmp/c5_$v.npz > $O/${TAG}_${v}_cmp5.txt 2>&1
done
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-per-step --no-cpu-baseline --config 5 --batch 8192 > $O/${TAG}_prod_${rep}.json 2> $O/${TAG}_prod_${rep}.err || exit $?
  for v in "$@"; do
    NMPC_LIB=$PWD/variants/$v.so timeout -k 10 300 python -u bench.py --no-per-step --no-cpu-baseline --config 5 --batch 8192 > $O/${TAG}_${v}_${rep}.json 2> $O/${TAG}_${v}_${rep}.err || exit $?
  done
done
echo ab5 done
