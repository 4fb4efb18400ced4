set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 60 ./tools_bin/qd_probe > $O/r06d_qd_probe.txt 2>&1 || echo "probe rc=$?"
timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_prod.npz > $O/r06d_prod_dump.log 2>&1 || exit $?
for v in nofdiv log; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_$v.npz > $O/r06d_${v}_dump.log 2>&1 || exit $?
done
python scripts/ab_bitwise.py --compare /tmp/ab_prod.npz /tmp/ab_nofdiv.npz > $O/r06d_prod_vs_nofdiv.txt 2>&1
python scripts/ab_bitwise.py --compare /tmp/ab_nofdiv.npz /tmp/ab_log.npz > $O/r06d_nofdiv_vs_log.txt 2>&1
echo dumps done
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --tb=short --timeout 300 --timeout-method thread > $O/r06d_tests.log 2>&1
echo "tests rc=$?"
