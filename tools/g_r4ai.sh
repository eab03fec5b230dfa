# Single calls reading their inputs from the pinned mirror (mi) vs the copy kernel (base):
# matcher parity on mi, then the drop-in rows interleaved.
set -o pipefail
ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_mi.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_posed.py > gpurun_out/r04ai_pytest_mi.log 2>&1 || exit 1
for i in 1 2; do
for v in base mi; do
  if [ "$v" = "base" ]; then lib=""; else lib="ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so"; fi
  env $lib timeout -k 10 400 python bench.py --rows --reps 20 > gpurun_out/r04ai_rows_$v$i.json 2> gpurun_out/r04ai_rows_$v$i.err || exit 2
  python3 -c "
import json; t=open('gpurun_out/r04ai_rows_$v$i.json').read(); d=json.loads([l for l in t.splitlines() if l.startswith('{')][-1])
print('$v$i', [(r['row'], r.get('lib_ms'), r.get('speedup_lib'), r['bit_exact']) for r in d['rows'] if r.get('lib_ms')])" || exit 3
done; done
echo ok
