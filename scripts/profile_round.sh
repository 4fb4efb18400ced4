#!/bin/bash
# rocprofv3 passes for the driver-style bench command (fused closed loop, K=20, W=5),
# run on the GPU box:
#   stats:  --kernel-trace --stats (CSV)            -> gpurun_out/prof_<tag>_stats/
#   pmc:    FETCH_SIZE | WRITE_SIZE | TCC hit/miss | SQ wave states (separate passes)
# then scripts/rocpd_summary.py --csv writes gpurun_out/<tag>_pmc.csv (timed dispatch per
# kernel) with each pass's bench line (steps, warmup, batch, I_bar, HIP-event kernel ms),
# so every roofline field of the bench line can be recomputed from profiles/.
# usage: [BENCH_ARGS="--config 5 --batch 8192"] scripts/profile_round.sh <tag>
set -e
set -o pipefail
TAG=${1:-r02}
R=$PWD
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-cpu-baseline --no-per-step --no-config5 --warmup 5 ${BENCH_ARGS:-}"
O=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_stats -o run -- python3 $B > $O/prof_${TAG}_stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_${TAG}_fetch -o run -- python3 $B > $O/prof_${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_${TAG}_write -o run -- python3 $B > $O/prof_${TAG}_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/prof_${TAG}_l2 -o run -- python3 $B > $O/prof_${TAG}_l2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU -d $O/prof_${TAG}_sq -o run -- python3 $B > $O/prof_${TAG}_sq.log 2>&1
cd $R && python3 scripts/rocpd_summary.py --csv $O/${TAG}_pmc.csv $O/prof_${TAG}_fetch $O/prof_${TAG}_write $O/prof_${TAG}_l2 $O/prof_${TAG}_sq > $O/${TAG}_pmc_summary.txt
# the rocpd databases stay on the box (gpurun copies back at most 64 MiB); the summary CSV
# and the pass logs (bench lines) come back
rm -rf $O/prof_${TAG}_fetch $O/prof_${TAG}_write $O/prof_${TAG}_l2 $O/prof_${TAG}_sq
find $O/prof_${TAG}_stats -name "*.db" -delete 2>/dev/null || true
echo profile done
