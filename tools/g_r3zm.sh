# host-fed leg (per-lane upload streams) at configs[1] and configs[4], then the bench lines.
set -o pipefail
mkdir -p gpurun_out
for w in tum tum5k; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --steps 30 \
      --parity-frames 8 > gpurun_out/r3zm.json 2>gpurun_out/r3zm.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r3zm.json')); print('$w', d['value'], d['parity']['bit_exact'], d['host_fed'], flush=True)" || exit 1
done
