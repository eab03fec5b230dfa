# List sizes (kTopK, kLaneTopK) against the configs[4] re-scoring: stamps per variant, then
# interleaved pipelined A/B.
set -o pipefail
for v in base t16 l8 t16l8; do
  if [ "$v" = "base" ]; then lib=""; else lib="ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so"; fi
  env $lib ORBX_MATCH_STAMPS=1 timeout -k 10 300 python bench.py --workload tum5k --steps 1 --warmup 1 --no-cpu-baseline --no-pipeline --parity-frames 16 > gpurun_out/r04w_st_$v.json 2> gpurun_out/r04w_st_$v.err || exit 1
  echo "$v $(grep 'seq stamps' gpurun_out/r04w_st_$v.err | tail -1)"
done
STEPS=20 bash tools/ab_lib.sh 2 tum5k base t16 l8 t16l8 || exit 2
STEPS=20 bash tools/ab_lib.sh 1 tum base t16 l8 t16l8 || exit 3
echo ok
