# round-6 GPU pass: -m gpu suite, smoke, the default bench line (with its config-5 leg), then
# a same-box A/B of the in-tree product against variants/<v>.so: alternating config-3 bench
# runs, one config-5 run and one work-bound run (16,384 scenarios) each.
# usage: scripts/r06_run.sh <tag> [variant...]   (logs under gpurun_out/)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=$1; shift
timeout -k 10 60 ./tools_bin/fp64_probe > $O/${TAG}_fp64_probe.txt 2>&1 || echo "probe rc=$?"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --tb=short --timeout 300 --timeout-method thread > $O/${TAG}_tests.log 2>&1
  rc=$?
  echo "tests rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit $?
  timeout -k 10 400 python -u bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit $?
  echo bench done
fi
for rep in ${AB_REPS:-1 2}; do
  timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --no-config5 > $O/${TAG}_prod_${rep}.json 2> $O/${TAG}_prod_${rep}.err || exit $?
  for v in "$@"; do
    NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --no-config5 > $O/${TAG}_${v}_${rep}.json 2> $O/${TAG}_${v}_${rep}.err || exit $?
  done
done
timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --config 5 --batch 8192 > $O/${TAG}_prod_c5.json 2> $O/${TAG}_prod_c5.err || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --config 5 --batch 8192 > $O/${TAG}_${v}_c5.json 2> $O/${TAG}_${v}_c5.err || exit $?
done
timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --no-config5 --batch 16384 > $O/${TAG}_prod_wb.json 2> $O/${TAG}_prod_wb.err || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-per-step --no-cpu-baseline --no-config5 --batch 16384 > $O/${TAG}_${v}_wb.json 2> $O/${TAG}_${v}_wb.err || exit $?
done
echo "all done"
