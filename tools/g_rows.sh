# Per-row drop-in calls and the other workloads' bench lines (round-2 refresh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --rows > gpurun_out/rows.json 2> gpurun_out/rows.err || { tail -5 gpurun_out/rows.err; exit 1; }
for w in tum5k kitti euroc; do
  timeout -k 10 300 python bench.py --workload $w > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || { tail -5 gpurun_out/b_$w.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b_$w.json')); print('$w', d['value'], d['unit'], d['ms_per_step'], d['parity'].get('bit_exact'), d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"
done
