# Dev: same-box A/B of several variant libraries: for each, the bench line, a work-bound
# batch (16,384 scenarios: per-iteration time = kernel time / work per slot), the longest
# chain alone and a bitwise output dump (scripts/ab_bitwise.py); logs under gpurun_out/ab_*
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for v in "$@"; do
  L=$PWD/variants/$v.so
  NMPC_LIB=$L timeout -k 10 300 python -u bench.py --no-per-step --no-cpu-baseline > $O/ab_${v}_bench.json 2> $O/ab_${v}_bench.err || exit $?
  NMPC_LIB=$L timeout -k 10 300 python -u bench.py --no-per-step --no-cpu-baseline --batch 16384 > $O/ab_${v}_b16k.json 2> $O/ab_${v}_b16k.err || exit $?
  NMPC_LIB=$L timeout -k 10 200 python -u scripts/chain_trace.py 2284 > $O/ab_${v}_chain.log 2>&1 || exit $?
  [ -n "$AB_DUMP" ] && { NMPC_LIB=$L AB_K=20 timeout -k 10 200 python -u scripts/ab_bitwise.py $O/ab_${v}.npz > $O/ab_${v}_dump.log 2>&1 || exit $?; }
done
echo ab done
