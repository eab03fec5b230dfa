# configs[4] with and without the matcher (the matcher's share of the pipelined step).
set -o pipefail
for i in 1 2; do
for a in "" "--no-match"; do
timeout -k 10 200 python bench.py --workload tum5k --no-cpu-baseline --no-local-map --no-host-fed --steps 20 --parity-frames 16 $a > gpurun_out/r04x.json 2> gpurun_out/r04x.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r04x.json')); print('tum5k [$a]', d['value'], d['ms_per_step'], d['roofline']['stage_ms'])" || exit 1
done; done
echo ok
