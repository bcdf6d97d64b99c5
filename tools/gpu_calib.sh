# FETCH_SIZE / WRITE_SIZE calibration on known access shapes (tools/fetch_calib.hip).
set -eu
TAG=${1:?tag}
mkdir -p gpurun_out
export TMPDIR=/tmp
B=tools/fetch_calib
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_calib_fetch -- $B > gpurun_out/${TAG}_calib_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_calib_write -- $B > gpurun_out/${TAG}_calib_write.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_calib_trace -- $B > gpurun_out/${TAG}_calib_trace.log 2>&1
python3 tools/fetch_calib_report.py gpurun_out/${TAG}_calib gpurun_out/${TAG}_fetch_calibration.json
echo calib done
