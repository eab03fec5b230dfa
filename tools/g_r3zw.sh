# Replay entry pick from registers (a: default) vs from LDS (b: ORBX_REPLAY_LDS_PICK=1):
# matcher tests on the default build, then the drop-in rows and the pipelined configs[1] /
# configs[4] benches, interleaved, two rounds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_posed.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3zw_pytest.log 2>&1 || { tail -5 gpurun_out/r3zw_pytest.log; exit 1; }
tail -1 gpurun_out/r3zw_pytest.log
for i in 1 2; do
  for v in a b; do
    L=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so
    ORBX_LIB=$L timeout -k 10 300 python bench.py --rows --reps 30 > gpurun_out/r3zw_rows_$v.json 2> gpurun_out/r3zw_rows_$v.err || exit 1
    python3 -c "
import json;d=json.load(open('gpurun_out/r3zw_rows_$v.json'))
print('$v rows', [(r['row'], r.get('lib_ms'), r['bit_exact']) for r in d['rows'] if r['row'] in ('a11','a12','a13','a14')], flush=True)" || exit 1
    for w in tum tum5k; do
      ORBX_LIB=$L timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --no-host-fed \
          --steps 50 --parity-frames 16 > gpurun_out/r3zw.json 2>gpurun_out/r3zw.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3zw.json')); s=d['roofline']['stage_ms']; print('$v $w', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['match'], flush=True)" || exit 1
    done
  done
done
