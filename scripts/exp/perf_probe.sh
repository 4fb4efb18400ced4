# Per-wave latency and per-phase cycle breakdown (run on the GPU box; needs the
# stamps build next to the product library).  usage: scripts/perf_probe.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-probe}
O=gpurun_out
ST=mpc-implementation_amd/nmpc_amd/libnmpc_amd_stamps.so
timeout -k 10 120 python -u scripts/lat_probe.py > $O/${T}_lat.log 2>&1 &&
timeout -k 10 120 env NMPC_LIB=$ST python -u scripts/phase_profile.py 3 1024 > $O/${T}_phase1024.log 2>&1 &&
timeout -k 10 120 env NMPC_LIB=$ST python -u scripts/phase_profile.py 3 4096 > $O/${T}_phase4096.log 2>&1 &&
timeout -k 10 120 env NMPC_LIB=$ST python -u scripts/resto_profile.py 256 > $O/${T}_resto256.log 2>&1 &&
timeout -k 10 120 python -u scripts/chain_stats.py > $O/${T}_chain.log 2>&1
