# round-6 config-5 A/B of the in-tree product against variants/<v>.so: bitwise config-5 and
# config-3 dumps, then alternating config-5 bench runs (8,192 scenarios)
# usage: scripts/r06_ab5.sh <tag> <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=$1; shift
AB_CONFIG=5 AB_B=1024 AB_K=5 timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab5_prod.npz > $O/${TAG}_prod_dump5.log 2>&1 || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so AB_CONFIG=5 AB_B=1024 AB_K=5 timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab5_$v.npz > $O/${TAG}_${v}_dump5.log 2>&1 || exit $?
  python scripts/ab_bitwise.py --compare /tmp/ab5_prod.npz /tmp/ab5_$v.npz > $O/${TAG}_${v}_cmp5.txt 2>&1
done
echo dumps done
for rep in ${AB_REPS:-1 2 3}; do
  timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --config 5 --batch 8192 > $O/${TAG}_prod_c5_${rep}.json 2> $O/${TAG}_prod_c5_${rep}.err || exit $?
  for v in "$@"; do
    NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --config 5 --batch 8192 > $O/${TAG}_${v}_c5_${rep}.json 2> $O/${TAG}_${v}_c5_${rep}.err || exit $?
  done
done
echo "all done"
