# configs[4]: levels per pyramid segment (ORBX_PZ_SEG; 8 = default: 0-7 + 7-11; 7: 0-6 + 6-11;
# 6: 0-5 + 5-10 + 10-11), pipelined, interleaved, two rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for sg in 8 7 6; do
    ORBX_PZ_SEG=$sg timeout -k 10 200 python bench.py --workload tum5k --no-cpu-baseline --no-local-map --no-host-fed \
        --steps 50 --parity-frames 16 > gpurun_out/r3zv.json 2>gpurun_out/r3zv.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3zv.json')); s=d['roofline']['stage_ms']; print('seg $sg', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['pyramid'], s['describe'], s['total'], s['match'], flush=True)" || exit 1
  done
done
