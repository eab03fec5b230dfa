# Pyramid segments at configs[4], extraction only (--no-match), A/B two rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in 8 0; do
    ORBX_PZ_SEG=$v timeout -k 10 200 python bench.py --workload tum5k --no-match --no-cpu-baseline --no-local-map --no-host-fed \
        --steps 50 --parity-frames 16 > gpurun_out/r3zo.json 2>gpurun_out/r3zo.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3zo.json')); print('tum5k extract-only seg $v', d['value'], d['ms_per_step'], d['parity']['bit_exact'], d['roofline']['stage_ms'], flush=True)" || exit 1
  done
done
