set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
L=$PWD/diag_stamps_tmp.so
NMPC_LIB=$L timeout -k 10 200 python -u scripts/phase_profile.py 3 1024 > $O/p1_phase.log 2>&1 || exit $?
NMPC_LIB=$L timeout -k 10 200 python -u scripts/resto_profile.py 1024 > $O/p1_resto.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/chain_trace.py 2284 > $O/p1_chain.log 2>&1 || exit $?
echo probe done
