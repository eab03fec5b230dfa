# Per-phase stamps and scoring counts of the sequence matcher (a -DORBX_DEBUG=1
# -DORBX_SCORE_COUNT=1 build, python -m orbslam2commentedbyxcm_amd.build --variant TAG ...).
# usage: bash tools/match_counts.sh TAG WORKLOAD  ->  gpurun_out/mcount_TAG_WL.err
set -o pipefail
TAG=$1; WL=${2:-tum5k}
mkdir -p gpurun_out
ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$TAG.so ORBX_MATCH_STAMPS=1 timeout -k 10 300 python bench.py \
    --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --parity-frames 0 --no-local-map --no-host-fed \
    > gpurun_out/mcount_${TAG}_${WL}.json 2> gpurun_out/mcount_${TAG}_${WL}.err || exit 1
grep -E "orbx (seq stamps|score counts)" gpurun_out/mcount_${TAG}_${WL}.err | tail -4
