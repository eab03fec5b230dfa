# Matcher footprint modes after the flat-load fix: 5 (lean split) vs 2 (three split launches),
# pipelined, configs[4] and configs[1], interleaved.
set -o pipefail
for i in 1 2; do
  for w in tum5k tum; do
    for m in 5 2; do
      ORBX_MATCH_MODE=$m timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --no-host-fed \
          --steps 20 --parity-frames 16 > gpurun_out/r4z.json 2>gpurun_out/r4z.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r4z.json')); s=d['roofline']['stage_ms']; print('$w mode $m', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['total'], s['match'], flush=True)" || exit 1
    done
  done
done
echo ok
