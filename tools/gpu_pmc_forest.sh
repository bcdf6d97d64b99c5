# rocprofv3 PMC passes of bench_forest.py (one counter group per pass, no traces beside them),
# summarised into gpurun_out/<tag>_pmc_kernels.json.
# usage: bash tools/gpu_pmc_forest.sh <tag> [bench_forest.py args]
set -eu
TAG=${1:?tag}
shift
ARGS=${*:---model bench_assets/rf_deployed.npz --rows 4000000 --steps 1 --warmup 0}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <suffix> <counters...>
    local s=$1; shift
    timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${TAG}_pmc$s -- python3 bench_forest.py $ARGS \
        > gpurun_out/${TAG}_pmc$s.log 2>&1 || { echo "pmc pass $s failed"; tail -5 gpurun_out/${TAG}_pmc$s.log; exit 1; }
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
run b SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run c FETCH_SIZE
run d WRITE_SIZE
python3 tools/pmc_summary.py --json gpurun_out/${TAG}_pmc_kernels.json gpurun_out/${TAG}_pmc
echo pmc done
