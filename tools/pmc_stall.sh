# Where the extraction kernels' wave cycles go: SQ_WAVE_CYCLES split into ACTIVE_INST_ANY /
# WAIT_INST_ANY (issue stalls) / WAIT_ANY (waitcnt, barrier), plus VALU-active cycles and
# the LDS array's busy and bank-conflict cycles (MI355X_MICROARCH.md, PMC table), one
# rocprofv3 --pmc pass (8 SQ counters, no traces) over the non-pipelined bench.
# usage: bash tools/pmc_stall.sh TAG [WORKLOAD]   ->  python tools/pmc_stall.py TAG
set -o pipefail
TAG=${1:-run}
WL=${2:-tum}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/${TAG}_stall -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline --parity-frames 0 --no-local-map --no-host-fed --workload $WL > $R/gpurun_out/${TAG}_stall.log 2>&1
rc=$?
echo "pmc_stall rc=$rc"
exit $rc
