# Vector-issue counters per kernel launch: SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_INSTS_LDS /
# SQ_WAVES in one rocprofv3 --pmc pass (counters only, no traces), summarised into
# profiles/<TAG>_<WORKLOAD>_pmc_valu.json by `python tools/pmc_valu.py <TAG>_<WORKLOAD>`.
# usage: bash tools/pmc_valu.sh TAG [WORKLOAD]   (bench.py --workload, default tum)
set -o pipefail
TAG=${1:-run}
WL=${2:-tum}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $R/gpurun_out/${TAG}_${WL}_valu -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-local-map --no-host-fed --parity-frames 0 --workload $WL > $R/gpurun_out/${TAG}_${WL}_valu.log 2>&1
rc=$?
echo "pmc_valu rc=$rc"
exit $rc
