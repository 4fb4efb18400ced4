# copy a round-5 measurement (scripts/r05_measure.sh + r05_measure2.sh, tag $1) from
# gpurun_out/ into profiles/ (run here, after the GPU calls)
T=${1:-r05}
O=gpurun_out; P=profiles
cp $O/prof_${T}_stats/run_kernel_stats.csv $P/${T}_kernel_stats.csv
cp $O/prof_${T}_stats/run_kernel_trace.csv $P/${T}_kernel_trace.csv
cp $O/${T}_pmc.csv $P/${T}_pmc.csv
tail -1 $O/${T}_bench.json > $P/${T}_bench.json
grep "^{" $O/prof_${T}_stats.log | tail -1 > $P/${T}_profiled_bench.json
cp $O/${T}_chain_trace.txt $P/${T}_chain_trace.txt
cp $O/${T}_step_times.txt $P/${T}_step_times.txt
(echo "# config 3, all 4,096 scenarios (regular-iteration phase profile; stamps build)"; cat $O/${T}_phases.txt
 echo; echo "# the bounding chain (scenario 2284), per-phase cycles"; cat $O/${T}_chain_phases.txt
 echo; echo "# the bounding chain, restoration line-search slots (NMPC_RESTO_TRIAL_STAMPS: barrier = trial_resto cycles, ftb = SOC block cycles, dual_ftb = trials)"; cat $O/${T}_chain_rphases.txt
 echo; echo "# the bounding chain, parts of a restoration iteration (NMPC_XSTAMPS, scripts/chain_xphases.py)"; cat $O/${T}_chain_xphases.txt
 echo; echo "# restoration line-search profile"; cat $O/${T}_resto_ls.txt) | grep -v amdgpu.ids > $P/${T}_phases.txt
cp $O/${T}_cfg5_pmc.csv $P/${T}_cfg5_pmc.csv
cp $O/prof_${T}_cfg5_stats/run_kernel_stats.csv $P/${T}_cfg5_kernel_stats.csv
cp $O/prof_${T}_cfg5_stats/run_kernel_trace.csv $P/${T}_cfg5_kernel_trace.csv
tail -1 $O/${T}_cfg5_bench.json > $P/${T}_cfg5_bench.json
grep "^{" $O/prof_${T}_cfg5_stats.log | tail -1 > $P/${T}_cfg5_profiled_bench.json
echo collected
