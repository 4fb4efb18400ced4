# round-6 phase measurements (diagnostic builds under variants/): the bounding chain's
# per-phase cycles, its restoration line search, the regular-iteration phase profile
cd $GRAFT_REPO_ROOT
O=gpurun_out; TAG=${1:-r06p}
NMPC_LIB=$PWD/variants/stamps.so timeout -k 10 120 python -u scripts/chain_phases.py > $O/${TAG}_chain_phases.txt 2>&1 || exit 1
NMPC_LIB=$PWD/variants/rstamps.so RESTO_TRIAL=1 timeout -k 10 120 python -u scripts/chain_phases.py > $O/${TAG}_chain_rphases.txt 2>&1 || exit 1
NMPC_LIB=$PWD/variants/stamps.so timeout -k 10 120 python -u scripts/phase_profile.py 3 4096 > $O/${TAG}_phases.txt 2>&1 || exit 1
NMPC_LIB=$PWD/variants/rstamps.so timeout -k 10 120 python -u scripts/resto_ls_profile.py 4096 > $O/${TAG}_resto_ls.txt 2>&1 || exit 1
NMPC_LIB=$PWD/variants/xst.so timeout -k 10 120 python -u scripts/chain_xphases.py > $O/${TAG}_chain_xphases.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/step_times.py $O/${TAG}_step_times.npz > $O/${TAG}_step_times.txt 2>&1 || exit 1
echo phases done
