# Replay width of the single drop-in calls: the row bench under ORBX_REPLAY_THREADS=64 / 256 / 1024.
set -o pipefail
mkdir -p gpurun_out
for rt in 64 256 1024; do
  ORBX_REPLAY_THREADS=$rt timeout -k 10 300 python bench.py --rows > gpurun_out/r3z_rows_$rt.json 2> gpurun_out/r3z_rows_$rt.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r3z_rows_$rt.json'))
for r in d['rows']:
    print('$rt', r['row'], r['size'][:22], r.get('lib_ms'), r['cpu_ms'], r.get('speedup_lib'), r['bit_exact'])
" || exit 1
done
