# configs[4] at the deep-pyramid lane offset: matcher stream priority (ORBX_MATCH_STREAM_PRIO 0 / -1), two rounds.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for pr in 0 -1; do
    ORBX_MATCH_STREAM_PRIO=$pr timeout -k 10 200 python bench.py --workload tum5k --no-cpu-baseline --no-local-map --no-host-fed \
        --steps 50 --parity-frames 16 > gpurun_out/r3zzb.json 2>gpurun_out/r3zzb.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3zzb.json')); s=d['roofline']['stage_ms']; print('prio $pr', d['value'], d['ms_per_step'], d['parity']['bit_exact'], s['total'], s['match'], flush=True)" || exit 1
  done
done
