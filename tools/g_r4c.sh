# Where the configs[1] step goes: extraction only, stages alone (one lane, not pipelined), default.
set -o pipefail
for a in "--no-match" "--no-pipeline --lanes 1" "--no-match --lanes 1" "" ; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-local-map --no-host-fed --steps 50 --parity-frames 0 $a > gpurun_out/r4c.json 2> gpurun_out/r4c.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r4c.json')); s=d['roofline']['stage_ms']; print('[$a]', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in s.items()}, flush=True)" || exit 1
done
for a in "--no-match" "--no-pipeline --lanes 1" "--no-match --lanes 1"; do
  timeout -k 10 200 python bench.py --workload tum5k --no-cpu-baseline --no-local-map --no-host-fed --steps 30 --parity-frames 0 $a > gpurun_out/r4c.json 2> gpurun_out/r4c.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r4c.json')); s=d['roofline']['stage_ms']; print('tum5k [$a]', d['value'], d['ms_per_step'], {k: round(x, 3) for k, x in s.items()}, flush=True)" || exit 1
done
