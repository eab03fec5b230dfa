# Timed-region length: the default 20 steps / 5 warmup against 100 / 50 (configs[1], configs[4]).
set -o pipefail
mkdir -p gpurun_out
for w in tum tum5k; do
  for i in 1 2; do
    for sw in "20 5" "100 50" "200 100"; do
      set -- $sw
      timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-host-fed --no-local-map --steps $1 --warmup $2 \
          --parity-frames 8 > gpurun_out/r3zh.json 2>gpurun_out/r3zh.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3zh.json')); print('$w steps $1 warmup $2', d['value'], d['ms_per_step'], flush=True)" || exit 1
    done
  done
done
