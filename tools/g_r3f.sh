# Replay phase stamps (k_proj_search lean form, replay inside the scoring workgroup, alone)
# for the replay variants a / b / c at configs[4] and configs[1].
set -o pipefail
mkdir -p gpurun_out
for w in tum5k tum; do
  for v in a b c; do
    ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so ORBX_MATCH_STAMPS=1 ORBX_MATCH_MODE=4 timeout -k 10 150 \
        python bench.py --workload $w --no-pipeline --no-cpu-baseline --no-local-map --parity-frames 0 --steps 3 --warmup 1 \
        > gpurun_out/r3f_$w$v.json 2> gpurun_out/r3f_$w$v.err || exit 1
    echo "$w $v"; grep stamps gpurun_out/r3f_$w$v.err | tail -1
  done
done
