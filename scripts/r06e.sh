# bisection of the qd() groups: bitwise dumps of single-group variants against nofdiv
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
NMPC_LIB=$PWD/variants/nofdiv.so timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_nofdiv.npz > $O/r06e_nofdiv_dump.log 2>&1 || exit $?
for v in ${VARS:-g1 g2 g3}; do
  NMPC_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_$v.npz > $O/r06e_${v}_dump.log 2>&1 || exit $?
  python scripts/ab_bitwise.py --compare /tmp/ab_nofdiv.npz /tmp/ab_$v.npz > $O/r06e_${v}_cmp.txt 2>&1
done
echo done
