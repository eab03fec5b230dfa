# Kernel-trace stats of the non-pipelined bench (matcher kernels run alone) per matcher mode.
# usage: bash tools/prof_modes.sh TAG MODE...
set -o pipefail
TAG=$1; shift
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  ORBX_MATCH_MODE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_m$m -o run -- \
      python $R/bench.py --no-pipeline --steps 10 --warmup 2 --no-cpu-baseline --parity-frames 0 > $R/gpurun_out/${TAG}_m$m.log 2>&1 || exit 1
done
