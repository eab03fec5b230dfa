# k_describe A/B: parity of variant b on the extraction tests, then the pipelined bench of
# a (HEAD) and b per workload with the describe stage's event time.
set -o pipefail
mkdir -p gpurun_out
VARIANTS=${VARIANTS:-"a b"}
PAR=${PAR:-b}
for v in $PAR; do
ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_extract.py \
    tests/test_gpu_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3v_pytest_$v.log 2>&1
rc=$?; echo "parity $v"; tail -1 gpurun_out/r3v_pytest_$v.log
if [ $rc -ne 0 ]; then exit $rc; fi
done
for w in tum5k tum; do
  for i in 1 2; do
    for v in $VARIANTS; do
      ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --workload $w \
          --no-cpu-baseline --no-local-map --no-host-fed --steps 30 --parity-frames 64 > gpurun_out/r3v.json 2>gpurun_out/r3v.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3v.json')); s=d['roofline']['stage_ms']; print('$w $v', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['describe'], s['total'], round(s['match'],4), flush=True)" || exit 1
    done
  done
done
