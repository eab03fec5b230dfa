# Scoring visit counts (diagnostics build) at configs[4] and configs[1].
set -o pipefail
for w in tum5k tum; do
  ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_cnt.so ORBX_MATCH_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline --no-pipeline --parity-frames 16 > gpurun_out/r04ab_$w.json 2> gpurun_out/r04ab_$w.err || exit 1
  echo "$w $(grep 'score counts' gpurun_out/r04ab_$w.err | tail -1)"
  echo "$w $(grep 'seq stamps' gpurun_out/r04ab_$w.err | tail -1)"
done
echo ok
