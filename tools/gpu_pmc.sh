# HBM traffic per kernel of the bench (rocprofv3 PMC, one counter group per pass; counters
# never share a pass with traces), summarised into gpurun_out/<tag>_pmc_kernels.json.
# usage: bash tools/gpu_pmc.sh <tag> [sq]     (sq: also the SQ instruction / LDS passes)
set -eu
TAG=${1:?tag}
mkdir -p gpurun_out
export TMPDIR=/tmp
A="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
run() {  # run <suffix> <counters...>
    local s=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${TAG}_pmc$s -- $A \
        > gpurun_out/${TAG}_pmc$s.log 2>&1 || { echo "pmc pass $s failed"; tail -5 gpurun_out/${TAG}_pmc$s.log; exit 1; }
}
run c FETCH_SIZE
run d WRITE_SIZE
if [ "${2:-}" = "sq" ]; then
    run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
    run b SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
fi
python3 tools/pmc_summary.py --json gpurun_out/${TAG}_pmc_kernels.json gpurun_out/${TAG}_pmc
echo pmc done
