# describe workgroups per CU (ORBX_DESC_LDS_EXTRA bytes of unused dynamic LDS) at configs[4] and configs[1].
set -o pipefail
mkdir -p gpurun_out
for w in tum5k tum; do
  for i in 1 2; do
    for ex in 0 14336 25600; do
      ORBX_DESC_LDS_EXTRA=$ex timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --no-host-fed \
          --steps 30 --parity-frames 16 > gpurun_out/r3zf.json 2>gpurun_out/r3zf.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3zf.json')); print('$w extra $ex', d['value'], d['ms_per_step'], d['parity']['bit_exact'], flush=True)" || exit 1
    done
  done
done
