# Arena host mirror coherent (base) vs non-coherent (anc), and the scoring merge's early
# exit (base) vs none (mx0): GPU tests on both variants, then drop-in rows and the
# pipelined configs[1] / configs[4] benches, interleaved.
set -o pipefail
for v in anc mx0; do
ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_posed.py tests/test_gpu_frame.py > gpurun_out/r04ad_pytest_$v.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_posed.py tests/test_gpu_pipeline.py > gpurun_out/r04ad_pytest_base.log 2>&1 || exit 1
for i in 1 2; do
for v in base anc mx0; do
  if [ "$v" = "base" ]; then lib=""; else lib="ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so"; fi
  env $lib timeout -k 10 400 python bench.py --rows --reps 20 > gpurun_out/r04ad_rows_$v$i.json 2> gpurun_out/r04ad_rows_$v$i.err || exit 2
  python3 -c "
import json; t=open('gpurun_out/r04ad_rows_$v$i.json').read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print('$v$i', [(r['row'], r.get('lib_ms'), r.get('speedup_lib'), r['bit_exact']) for r in d['rows'] if r.get('lib_ms')])" || exit 3
done; done
STEPS=20 bash tools/ab_lib.sh 2 tum base mx0 || exit 4
STEPS=20 bash tools/ab_lib.sh 2 tum5k base mx0 || exit 5
echo ok
