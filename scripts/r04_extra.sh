# Round-4 measurement pass (run on the box): config-5 rocprofv3 profile, the config-5
# bench line, per-phase cycles (stamps build), and the fused launch's step-time tail.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
STAMPS=$PWD/mpc-implementation_amd/nmpc_amd/libnmpc_amd_stamps.so
[ -n "$PROFILE_CFG5" ] && { BENCH_ARGS="--config 5 --batch 8192" bash scripts/profile_round.sh r04_cfg5 || exit $?; }
[ -z "$SKIP_CFG5" ] && { timeout -k 10 300 python -u bench.py --config 5 --batch 8192 --no-per-step > $O/r04_cfg5_bench.json 2> $O/r04_cfg5_bench.err || exit $?; }
{ echo "# 1) scripts/phase_profile.py 3 4096"; NMPC_LIB=$STAMPS timeout -k 10 200 python -u scripts/phase_profile.py 3 4096; } > $O/r04_phases.txt 2>&1 || exit $?
{ echo; echo "# 2) scripts/phase_profile.py 5 2048"; NMPC_LIB=$STAMPS timeout -k 10 200 python -u scripts/phase_profile.py 5 2048; } >> $O/r04_phases.txt 2>&1 || exit $?
{ echo; echo "# 3) scripts/resto_profile.py 4096 and 16"; NMPC_LIB=$STAMPS timeout -k 10 200 python -u scripts/resto_profile.py 4096; NMPC_LIB=$STAMPS timeout -k 10 200 python -u scripts/resto_profile.py 16; } >> $O/r04_phases.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/step_times.py > $O/r04_step_times.txt 2>&1 || exit $?
B=$(python - <<'PY'
import re
t = open("gpurun_out/r04_step_times.txt").read().split("latest-finishing scenarios")[1].splitlines()
print(next(int(m.group(1)) for l in t if (m := re.match(r"\s*(?:scenario\s*)?(\d+)\b", l))))
PY
) && timeout -k 10 120 python -u scripts/chain_trace.py $B > $O/r04_chain_trace.txt 2>&1 || exit $?
echo extra done
