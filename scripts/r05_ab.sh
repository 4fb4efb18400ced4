# round-5 same-box A/B of the in-tree product against variants/<v>.so: bitwise dumps
# (config 3 cold solve + 20-step closed loop; config 5, 1024 scenarios x 5 steps), then
# alternating config-3 bench runs and one work-bound run (16,384 scenarios) each
# usage: scripts/r05_ab.sh <tag> <variant>...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=$1; shift
timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_prod.npz > $O/${TAG}_prod_dump.log 2>&1 || exit $?
AB_CONFIG=5 AB_B=1024 AB_K=5 timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab5_prod.npz > $O/${TAG}_prod_dump5.log 2>&1 || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_$v.npz > $O/${TAG}_${v}_dump.log 2>&1 || exit $?
  python scripts/ab_bitwise.py --compare /tmp/ab_prod.npz /tmp/ab_$v.npz > $O/${TAG}_${v}_cmp.txt 2>&1
  NMPC_LIB=$PWD/variants/$v.so AB_CONFIG=5 AB_B=1024 AB_K=5 timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab5_$v.npz > $O/${TAG}_${v}_dump5.log 2>&1 || exit $?
  python scripts/ab_bitwise.py --compare /tmp/ab5_prod.npz /tmp/ab5_$v.npz > $O/${TAG}_${v}_cmp5.txt 2>&1
done
for rep in ${AB_REPS:-1 2}; do
  timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline > $O/${TAG}_prod_${rep}.json 2> $O/${TAG}_prod_${rep}.err || exit $?
  for v in "$@"; do
    NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline > $O/${TAG}_${v}_${rep}.json 2> $O/${TAG}_${v}_${rep}.err || exit $?
  done
done
timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --batch 16384 > $O/${TAG}_prod_wb.json 2> $O/${TAG}_prod_wb.err || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --batch 16384 > $O/${TAG}_${v}_wb.json 2> $O/${TAG}_${v}_wb.err || exit $?
done
echo ab done
# the bounding chain alone (trace on), product and variants
timeout -k 10 120 python -u scripts/chain_trace.py > $O/${TAG}_prod_chain.txt 2>&1 || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 120 python -u scripts/chain_trace.py > $O/${TAG}_${v}_chain.txt 2>&1 || exit $?
done
echo chains done
