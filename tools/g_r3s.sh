# Matcher change: parity, then scoring stamps and the pipelined A/B (a = new, c = HEAD).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_pipeline.py tests/test_gpu_posed.py \
    tests/test_gpu_fuse.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3s_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3s_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in tum5k tum; do
  for v in a c; do
    ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so ORBX_MATCH_STAMPS=1 ORBX_MATCH_MODE=4 timeout -k 10 150 \
        python bench.py --workload $w --no-pipeline --no-cpu-baseline --no-local-map --parity-frames 0 --steps 3 --warmup 1 \
        > gpurun_out/r3s_st.json 2> gpurun_out/r3s_st_$w$v.err || exit 1
    echo "$w $v"; grep stamps gpurun_out/r3s_st_$w$v.err | tail -1 | cut -c1-200
  done
done
for w in tum5k tum; do
  for i in 1 2; do
    for v in a c; do
      ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --workload $w \
          --no-cpu-baseline --no-local-map --steps 30 --parity-frames 64 > gpurun_out/r3s.json 2>gpurun_out/r3s.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3s.json')); print('$w $v', d['value'], d['ms_per_step'], d['parity']['bit_exact'], {k: round(x,4) for k,x in d['roofline']['stage_ms'].items()}, flush=True)"
    done
  done
done
