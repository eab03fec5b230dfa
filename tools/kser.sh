# Kernel trace of one bench shape (extra bench.py args after the tag), e.g. the serialised
# step (--no-pipeline --lanes 1) beside the pipelined one, for per-kernel durations alone.
# usage: bash tools/kser.sh WORKLOAD TAG [BENCH ARGS...]  ->  gpurun_out/kser_TAG_WL/run_kernel_stats.csv
set -o pipefail
WL=$1; TAG=$2; shift 2
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kser_${TAG}_${WL} -o run -- \
    python3 $R/bench.py --workload $WL --steps 10 --warmup 3 --no-cpu-baseline --parity-frames 0 --no-local-map \
    --no-host-fed "$@" > $R/gpurun_out/kser_${TAG}_${WL}.json 2> $R/gpurun_out/kser_${TAG}_${WL}.err || exit 1
echo "kser $WL $TAG ok"
