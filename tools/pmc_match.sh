# PMC counters of the bench step (extract + match) -- one counter group per pass.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmcm1 -o run -- $B > gpurun_out/pmcm1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmcm2 -o run -- $B > gpurun_out/pmcm2.log 2>&1
echo rc=$?
