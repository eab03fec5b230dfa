# Pyramid segments x matcher stream priority (ORBX_MATCH_STREAM_PRIO), pipelined, two rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in "tum5k 8 0" "tum5k 8 -1" "tum5k 0 0" "tum5k 0 -1" "tum 8 0" "tum 8 -1"; do
    set -- $v
    ORBX_PZ_SEG=$2 ORBX_MATCH_STREAM_PRIO=$3 timeout -k 10 200 python bench.py --workload $1 --no-cpu-baseline --no-local-map --no-host-fed \
        --steps 50 --parity-frames 16 > gpurun_out/r3zp.json 2>gpurun_out/r3zp.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3zp.json')); s=d['roofline']['stage_ms']; print('$v', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['pyramid'], s['total'], s['match'], flush=True)" || exit 1
  done
done
