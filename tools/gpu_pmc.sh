# PMC counters for the hot kernels (separate passes; counters cannot share a pass with traces).
set -u
mkdir -p gpurun_out
TAG=${1:-rx}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc_${TAG}a -- $A > gpurun_out/pmc_${TAG}a.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_${TAG}b -- $A > gpurun_out/pmc_${TAG}b.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_${TAG}c -- $A > gpurun_out/pmc_${TAG}c.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_${TAG}d -- $A > gpurun_out/pmc_${TAG}d.log 2>&1 || exit 1
echo pmc done
