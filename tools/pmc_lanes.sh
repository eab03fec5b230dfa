# VALU lane utilisation and instruction mix per kernel (one --pmc pass, serialised dispatches)
# under the driver-shaped bench: SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU) is the
# fraction of lanes active per VALU issue (divergence), with the VALU / SALU / branch / VMEM
# instruction counts beside it.
# usage: bash tools/pmc_lanes.sh TAG [WORKLOAD]  ->  python tools/pmc_lanes.py TAG
set -o pipefail
TAG=${1:-run}
WL=${2:-tum}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --parity-frames 0 --no-local-map --no-host-fed --workload $WL"
timeout -s KILL 150 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH \
    SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES --output-format csv -d $R/gpurun_out/${TAG}_lanes -o run -- $CMD \
    > $R/gpurun_out/${TAG}_lanes.log 2>&1 || { echo "lanes pass failed"; exit 1; }
echo "pmc_lanes ok"
