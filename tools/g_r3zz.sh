# configs[1]: lane offset stage (ORBX_LANE_OFFSET; 2 = default, after blur + FAST strength;
# 0 = lanes in step; 1 pyramid; 3 FAST cells; 4 octree), pipelined, interleaved, two rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for lo in 2 4 1 3; do
    ORBX_LANE_OFFSET=$lo timeout -k 10 200 python bench.py --workload tum --no-cpu-baseline --no-local-map --no-host-fed \
        --steps 50 --parity-frames 16 > gpurun_out/r3zy.json 2>gpurun_out/r3zy.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3zy.json')); s=d['roofline']['stage_ms']; print('offset $lo', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['total'], s['match'], flush=True)" || exit 1
  done
done
