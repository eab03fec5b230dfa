# Matcher host-call tests, then the drop-in rows: completion-word spin (default) against
# the stream synchronise (ORBX_CALL_SYNC=1), two rounds.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03q}
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_posed.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -5 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for i in 1 2; do
  for v in spin sync; do
    if [ $v = spin ]; then E="ORBX_X=0"; else E="ORBX_CALL_SYNC=1"; fi
    env $E timeout -k 10 300 python bench.py --rows --reps 30 > gpurun_out/${T}_rows_$v.json 2> gpurun_out/${T}_rows_$v.err || exit 1
    python3 -c "
import json;d=json.load(open('gpurun_out/${T}_rows_$v.json'))
for r in d['rows']:
    if r['row'] in ('a11','a12','a13','a14'): print('$v', r['row'], r['gpu_ms'], r.get('lib_ms'), r['cpu_ms'], r.get('speedup_lib'), r['bit_exact'], flush=True)" || exit 1
  done
done
