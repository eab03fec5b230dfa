# A/B timing of bench.py argument sets, interleaved over ROUNDS rounds (one process per run).
# usage: bash tools/ab_args.sh ROUNDS "ARGS1" "ARGS2" ...   (ARGS may start with ENV=V words;
#   ':' stands for a space inside one ARGS, for tools/gpu_job.sh's run= step)
set -o pipefail
N=$1; shift
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  j=0
  for a in "$@"; do
    a=${a//:/ }
    j=$((j+1))
    env $(echo "$a" | tr ' ' '\n' | grep '=' | tr '\n' ' ') timeout -k 10 200 python bench.py --no-cpu-baseline \
        --parity-frames 0 --steps 30 $(echo "$a" | tr ' ' '\n' | grep -v '=' | tr '\n' ' ') \
        > gpurun_out/abargs_$j$i.json 2>gpurun_out/abargs_$j$i.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/abargs_$j$i.json')); print('[$a]', d['value'], d['ms_per_step'], {k: round(x,4) for k,x in d['roofline']['stage_ms'].items()}, flush=True)"
  done
done
