set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  NMPC_LIB=$PWD/variants/$v.so AB_K=20 timeout -k 10 200 python -u scripts/ab_bitwise.py gpurun_out/ab_${v}.npz > gpurun_out/ab_${v}_dump.log 2>&1 || exit $?
done
echo done
