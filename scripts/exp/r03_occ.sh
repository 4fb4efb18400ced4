set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
export NMPC_LIB=$PWD/mpc-implementation_amd/nmpc_amd/libnmpc_amd_stamps.so
for cfg in "A - 1024" "A - 4096" "B 40960 1024" "B - 1024" "B - 2048" "B - 4096" "C 40960 1024" "C - 2048" "C - 4096"; do
  set -- $cfg
  if [ "$1" != "A" ]; then export NMPC_FORCE_CLASS=$1; else unset NMPC_FORCE_CLASS; fi
  if [ "$2" != "-" ]; then export NMPC_LDS_BYTES=$2; else unset NMPC_LDS_BYTES; fi
  timeout -k 10 120 python -u scripts/occupancy_probe.py $3 >> $O/r03c_occ.log 2>&1 || exit $?
done
echo occ done
