# Dev: bitwise comparison of variant libraries against the in-tree product library, plus
# a test file run with the first variant; text results under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_prod.npz > gpurun_out/ab_prod_dump.log 2>&1 || exit $?
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_${v}.npz > gpurun_out/ab_${v}_dump.log 2>&1 || exit $?
  python scripts/ab_bitwise.py --compare /tmp/ab_prod.npz /tmp/ab_${v}.npz > gpurun_out/ab_${v}_cmp.txt 2>&1
done
if [ -n "$TESTS" ]; then
  NMPC_LIB=$PWD/variants/$1.so timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread $TESTS > gpurun_out/ab_tests.log 2>&1
  echo "tests rc=$?"
fi
echo done
