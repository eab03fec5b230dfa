# The matcher started after lane 0 passes the lane-offset stage (ORBX_MATCH_AFTER_L0=1) vs
# after the batch's extraction alone, pipelined, interleaved.
set -o pipefail
for i in 1 2 3; do
  for w in tum5k tum; do
    for a in 0 1; do
      ORBX_MATCH_AFTER_L0=$a timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --no-host-fed \
          --steps 20 --parity-frames 16 > gpurun_out/r4ae.json 2>gpurun_out/r4ae.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r4ae.json')); s=d['roofline']['stage_ms']; print('$w after_l0=$a', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['total'], s['match'], flush=True)" || exit 1
    done
  done
done
echo ok
