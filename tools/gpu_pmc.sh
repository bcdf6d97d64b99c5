# PMC counters for the bench kernels (separate passes; counters never share a pass with traces).
set -u
mkdir -p gpurun_out
TAG=${1:-rx}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
run() {  # run <suffix> <counters...>
    local s=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_${TAG}$s -- $A \
        > gpurun_out/pmc_${TAG}$s.log 2>&1 || { echo "pmc pass $s failed"; exit 1; }
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
run b SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_COUNT
run c FETCH_SIZE
run d WRITE_SIZE
echo pmc done
