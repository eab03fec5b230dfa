# Compute-side PMC counters of the bench's kernels (one counter group per pass).
# usage: bash tools/pmc_kernel.sh TAG
set -o pipefail
TAG=${1:-run}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/${TAG}_k1 -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_k1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_k2 -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_k2.log 2>&1
rc=$?
echo "pmc_kernel rc=$rc"
exit $rc
