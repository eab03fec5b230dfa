# med3 sorted insertion in the scoring: matcher parity, stamps, interleaved A/B vs the old insert.
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_posed.py tests/test_gpu_pipeline.py > gpurun_out/r04y_pytest.log 2>&1 || exit 1
for v in base med0; do
  if [ "$v" = "base" ]; then lib=""; else lib="ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so"; fi
  env $lib ORBX_MATCH_STAMPS=1 timeout -k 10 300 python bench.py --workload tum5k --steps 1 --warmup 1 --no-cpu-baseline --no-pipeline --parity-frames 16 > gpurun_out/r04y_st_$v.json 2> gpurun_out/r04y_st_$v.err || exit 2
  echo "$v $(grep 'seq stamps' gpurun_out/r04y_st_$v.err | tail -1)"
done
STEPS=20 bash tools/ab_lib.sh 3 tum5k base med0 || exit 3
STEPS=20 bash tools/ab_lib.sh 2 tum base med0 || exit 4
echo ok
