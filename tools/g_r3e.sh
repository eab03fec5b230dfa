# Fixpoint replay: matcher parity tests, then A/B of the replay forms at configs[4] and configs[1]
# (a = fixpoint + single re-scoring, b = fixpoint + row-batched re-scoring, c = round replay).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_pipeline.py tests/test_gpu_posed.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3e_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in tum5k tum; do
  for i in 1 2; do
    for v in a b c; do
      ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --workload $w \
          --no-cpu-baseline --no-local-map --steps 30 --parity-frames 64 > gpurun_out/r3e_${w}_$v$i.json 2>gpurun_out/r3e_${w}_$v$i.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3e_${w}_$v$i.json')); print('$w $v', d['value'], d['ms_per_step'], d['parity']['bit_exact'], {k: round(x,4) for k,x in d['roofline']['stage_ms'].items()}, flush=True)"
    done
  done
done
