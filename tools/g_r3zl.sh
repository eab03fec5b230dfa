# k_pyramid level-0 tile size sweep (ORBX_PZ_TILE) at configs[4] and configs[1], two rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for t in ${TILES:-default 160x120 214x160 128x120 160x96}; do
    for w in tum5k tum; do
      if [ "$t" = default ]; then unset ORBX_PZ_TILE; else export ORBX_PZ_TILE=$t; fi
      timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --no-host-fed \
          --steps 50 --parity-frames 8 > gpurun_out/r3zl.json 2>gpurun_out/r3zl.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3zl.json')); print('$w $t', d['value'], d['ms_per_step'], d['parity']['bit_exact'], d['roofline']['stage_ms']['pyramid'], flush=True)" || exit 1
    done
  done
done
