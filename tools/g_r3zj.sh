# Sensitivity of configs[4] to the replay kernel's LDS (ORBX_COMMIT_LDS_EXTRA bytes of unused dynamic LDS).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for ex in 0 16384 32768; do
    ORBX_COMMIT_LDS_EXTRA=$ex timeout -k 10 200 python bench.py --workload tum5k --no-cpu-baseline --no-local-map --no-host-fed \
        --steps 50 --parity-frames 8 > gpurun_out/r3zj.json 2>gpurun_out/r3zj.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3zj.json')); print('tum5k extra $ex', d['value'], d['ms_per_step'], d['parity']['bit_exact'], flush=True)" || exit 1
  done
done
