# round-5 GPU pass: tests, bench, restoration line-search profile, raw step times
cd $GRAFT_REPO_ROOT
TAG=${1:-r05}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --tb=short --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
echo "tests rc $?" > gpurun_out/${TAG}_status.txt
timeout -k 10 150 python bench.py --no-per-step > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
if [ -f variants/librstamps.so ]; then
  NMPC_LIB=$PWD/variants/librstamps.so timeout -k 10 120 python scripts/resto_ls_profile.py 16 > gpurun_out/${TAG}_resto_ls.txt 2>&1 || exit 1
  NMPC_LIB=$PWD/variants/librstamps.so timeout -k 10 120 python scripts/resto_ls_profile.py 4096 >> gpurun_out/${TAG}_resto_ls.txt 2>&1 || exit 1
fi
timeout -k 10 200 python scripts/step_times.py gpurun_out/${TAG}_steptimes.npz > gpurun_out/${TAG}_step_times.txt 2>&1
