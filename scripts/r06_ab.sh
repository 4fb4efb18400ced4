# round-6 same-box A/B of the in-tree product against variants/<v>.so: bitwise dumps
# (config 3: cold solve + 20-step closed loop, 4,096 scenarios; config 5: 1,024 x 5), then
# the bounding chain alone, alternating config-3 bench runs, one config-5 run and one
# work-bound run (16,384 scenarios)
# usage: scripts/r06_ab.sh <tag> <variant>...
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
echo dumps done
# the bounding chain alone (trace on), product and variants
timeout -k 10 120 python -u scripts/chain_trace.py > $O/${TAG}_prod_chain.txt 2>&1 || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 120 python -u scripts/chain_trace.py > $O/${TAG}_${v}_chain.txt 2>&1 || exit $?
done
NO_TESTS=1 bash scripts/r06_run.sh $TAG "$@"
