# Matcher stream confined to every k-th CU (ORBX_MATCH_CUSTRIDE) at configs[4] and configs[1].
set -o pipefail
for i in 1 2; do
  for w in tum5k tum; do
    for k in 1 2 4; do
      ORBX_MATCH_CUSTRIDE=$k timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --no-host-fed \
          --steps 20 --parity-frames 16 > gpurun_out/r4aa.json 2>gpurun_out/r4aa.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r4aa.json')); s=d['roofline']['stage_ms']; print('$w custride $k', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['total'], s['match'], flush=True)" || exit 1
    done
  done
done
echo ok
