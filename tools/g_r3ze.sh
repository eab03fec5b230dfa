# Extraction lanes per batch (bench.py --lanes) at configs[1] and configs[4].
set -o pipefail
mkdir -p gpurun_out
for w in tum tum5k; do
  for ln in 2 3 4 2; do
    timeout -k 10 200 python bench.py --workload $w --lanes $ln --no-cpu-baseline --no-local-map --no-host-fed --steps 30 \
        --parity-frames 16 > gpurun_out/r3ze.json 2>gpurun_out/r3ze.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3ze.json')); print('$w lanes $ln', d['value'], d['ms_per_step'], d['parity']['bit_exact'], flush=True)" || exit 1
  done
done
