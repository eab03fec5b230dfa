# Kernel-trace A/B of library builds: one rocprofv3 --kernel-trace --stats run of the
# driver-shaped bench per build (20 timed steps), for per-kernel average durations.
# usage: bash tools/kprof_lib.sh WORKLOAD TAG1 TAG2 ...   (TAG as in tools/ab_lib.sh)
# read:  gpurun_out/kprof_TAG_WL/run_kernel_stats.csv
set -o pipefail
WL=$1; shift
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = "base" ]; then unset ORBX_LIB; else export ORBX_LIB=$R/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kprof_${v}_${WL} -o run -- \
      python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --workload $WL --no-cpu-baseline --parity-frames 0 \
      > $R/gpurun_out/kprof_${v}_${WL}.json 2> $R/gpurun_out/kprof_${v}_${WL}.err || exit 1
  echo "kprof $WL $v ok"
done
