# Matcher footprint modes (ORBX_MATCH_MODE, orbx_matcher_set_footprint) pipelined at
# configs[4] and configs[1], two rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for w in tum5k tum; do
    for m in 5 4 2 0; do
      ORBX_MATCH_MODE=$m timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --no-host-fed \
          --steps 50 --parity-frames 16 > gpurun_out/r3zq.json 2>gpurun_out/r3zq.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3zq.json')); s=d['roofline']['stage_ms']; print('$w mode $m', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['total'], s['match'], flush=True)" || exit 1
    done
  done
done
