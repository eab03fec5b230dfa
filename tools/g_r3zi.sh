# Timed-region length vs warmup: 20 steps after 5 / 100 warmup, 100 steps after 5 / 100 (configs[1]).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for sw in "20 5" "20 100" "100 5" "100 100"; do
    set -- $sw
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-fed --no-local-map --steps $1 --warmup $2 \
        --parity-frames 8 > gpurun_out/r3zi.json 2>gpurun_out/r3zi.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3zi.json')); print('tum steps $1 warmup $2', d['value'], d['ms_per_step'], flush=True)" || exit 1
  done
done
