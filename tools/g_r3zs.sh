# Every GPU test at HEAD, then the drop-in rows with the per-row replay width (a13 / a14
# at 1024 threads) against the one-wave replay for every row (ORBX_REPLAY_THREADS=64).
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03n}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  for v in row 64; do
    if [ $v = row ]; then E="ORBX_X=0"; else E="ORBX_REPLAY_THREADS=64"; fi
    env $E timeout -k 10 300 python bench.py --rows --reps 30 > gpurun_out/${T}_rows_$v.json 2> gpurun_out/${T}_rows_$v.err || exit 1
    python3 -c "
import json;d=json.load(open('gpurun_out/${T}_rows_$v.json'))
for r in d['rows']:
    if r['row'] in ('a11','a12','a13','a14'): print('$v', r['row'], r['gpu_ms'], r.get('lib_ms'), r['cpu_ms'], r.get('speedup_lib'), r['bit_exact'], flush=True)" || exit 1
  done
done
