# k_describe A/B, isolated: one lane, no pipeline, the describe stage's event time per
# variant (a = HEAD, b = packed-f32 sampling, c = + four keypoints per wave, d = four per
# wave with scalar sampling, e = float pattern, scalar sampling), then the
# pipelined bench again.
set -o pipefail
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"a b c"}
for v in ${PAR:-}; do
  ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_extract.py tests/test_gpu_pipeline.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3w_pytest_$v.log 2>&1
  rc=$?; echo "parity $v"; tail -1 gpurun_out/r3w_pytest_$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for w in ${WLS:-tum5k tum}; do
  for v in $VARIANTS; do
    ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --workload $w --lanes 1 --no-pipeline \
        --no-cpu-baseline --no-local-map --no-host-fed --steps 20 --parity-frames 0 > gpurun_out/r3w.json 2>gpurun_out/r3w.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3w.json')); s=d['roofline']['stage_ms']; print('iso $w $v', {k: round(x, 4) for k, x in s.items()}, flush=True)" || exit 1
  done
done
for w in ${WLS:-tum5k tum}; do
  for i in 1 2; do
    for v in $VARIANTS; do
      ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --workload $w \
          --no-cpu-baseline --no-local-map --no-host-fed --steps 30 --parity-frames 16 > gpurun_out/r3w.json 2>gpurun_out/r3w.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3w.json')); s=d['roofline']['stage_ms']; print('$w $v', d['value'], d['ms_per_step'], d['parity']['bit_exact'], flush=True)" || exit 1
    done
  done
done
