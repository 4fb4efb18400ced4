# FETCH_SIZE / WRITE_SIZE calibration passes (scripts/fetch_calib.hip); run on the GPU box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/calib_fetch -o run -- $R/scripts/fetch_calib > $R/gpurun_out/calib_fetch.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/calib_write -o run -- $R/scripts/fetch_calib > $R/gpurun_out/calib_write.log 2>&1
