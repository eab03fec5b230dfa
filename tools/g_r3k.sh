# Drop-in host calls: Python-side and in-library times.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --rows --reps 30 > gpurun_out/r3k_rows.json 2> gpurun_out/r3k_rows.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/r3k_rows.json'))
for r in d['rows']: print(r['row'], r['size'][:20], r['gpu_ms'], r.get('lib_ms'), r['cpu_ms'], r['speedup'], r.get('speedup_lib'), r['bit_exact'])"
