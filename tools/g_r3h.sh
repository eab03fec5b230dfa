# Pipeline depth and lane offset at configs[4] and configs[1] (interleaved A/B).
set -o pipefail
mkdir -p gpurun_out
for w in tum5k tum; do
  for i in 1 2; do
    for e in "ORBX_PIPE_NBUF=2" "ORBX_PIPE_NBUF=3" "ORBX_PIPE_NBUF=3 ORBX_LANE_OFFSET=1" "ORBX_PIPE_NBUF=4"; do
      env $e timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --steps 30 --parity-frames 64 \
          > gpurun_out/r3h.json 2>gpurun_out/r3h.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3h.json')); print('$w [$e]', d['value'], d['ms_per_step'], d['parity']['bit_exact'], {k: round(x,4) for k,x in d['roofline']['stage_ms'].items()}, flush=True)"
    done
  done
done
