# A/B timing of the pipelined bench (extract + match on two streams) under different environment settings.
# usage: bash tools/ab_pipe.sh ROUNDS "ENV1" "ENV2" ...   (each ENV is "K=V K2=V2" or "-")
set -o pipefail
N=$1; shift
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  j=0
  for e in "$@"; do
    j=$((j+1))
    if [ "$e" = "-" ]; then e=""; fi
    env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --parity-frames 0 > gpurun_out/abpipe_$j$i.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abpipe_$j$i.json')); print('[$e]', d['value'], {k: round(x,4) for k,x in d['roofline']['stage_ms'].items()})"
  done
done
