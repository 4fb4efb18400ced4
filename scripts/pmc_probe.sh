# Instruction-cache counters of the bench's closed-loop kernel (run on the GPU box)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-per-step"
PMC=${PMC:-"SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH"}
T=${1:-icache}
timeout -s KILL 200 rocprofv3 --pmc $PMC -d $R/gpurun_out/prof_$T -o run -- python3 $B > $R/gpurun_out/prof_$T.log 2>&1
cd $R && python3 scripts/rocpd_summary.py gpurun_out/prof_$T > gpurun_out/${T}_summary.txt 2>&1
