set -o pipefail
mkdir -p gpurun_out
ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_b.so timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g8.log 2>&1 || { tail -30 gpurun_out/g8.log; exit 1; }
tail -1 gpurun_out/g8.log
for v in a b; do for w in tum tum5k; do
  ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so ORBX_MATCH_MODE=4 ORBX_MATCH_STAMPS=1 timeout -k 10 150 python bench.py --workload $w --no-pipeline --no-cpu-baseline --parity-frames 0 --steps 3 --warmup 1 > gpurun_out/st.json 2> gpurun_out/st.err || exit 1
  echo "$v $w $(grep stamps gpurun_out/st.err | tail -1 | cut -c1-200)"
done; done
bash tools/ab_args.sh 2 "ORBX_LIB=orbslam2commentedbyxcm_amd/_ab/liborbx_a.so" "ORBX_LIB=orbslam2commentedbyxcm_amd/_ab/liborbx_b.so" "ORBX_LIB=orbslam2commentedbyxcm_amd/_ab/liborbx_a.so --workload tum5k" "ORBX_LIB=orbslam2commentedbyxcm_amd/_ab/liborbx_b.so --workload tum5k"
