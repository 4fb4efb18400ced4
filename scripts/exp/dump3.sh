# Dev: bitwise comparison of variant libraries against a reference dump (variants/ab_base.npz);
# only the comparison text comes back (gpurun_out/ab_<v>_cmp.txt)
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so AB_K=20 timeout -k 10 200 python -u scripts/ab_bitwise.py /tmp/ab_${v}.npz > gpurun_out/ab_${v}_dump.log 2>&1 || exit $?
  python scripts/ab_bitwise.py --compare variants/ab_base.npz /tmp/ab_${v}.npz > gpurun_out/ab_${v}_cmp.txt 2>&1
done
echo done
