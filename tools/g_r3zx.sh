# configs[4]: extraction lanes per step (2 = default), pipelined, interleaved, two rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for ln in 2 3 4; do
    timeout -k 10 200 python bench.py --workload tum5k --lanes $ln --no-cpu-baseline --no-local-map --no-host-fed \
        --steps 50 --parity-frames 16 > gpurun_out/r3zx.json 2>gpurun_out/r3zx.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3zx.json')); s=d['roofline']['stage_ms']; print('lanes $ln', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['total'], s['match'], flush=True)" || exit 1
  done
done
