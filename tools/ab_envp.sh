# A/B of environment settings in the pipelined bench (the driver's step shape), interleaved.
# usage: bash tools/ab_envp.sh ROUNDS WORKLOAD "ENV1" "ENV2" ...   (each ENV "K=V K2=V2" or "-")
# STEPS (default 50) and EXTRA (more bench.py args) from the environment.
set -o pipefail
N=$1; WL=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for e in "$@"; do
    if [ "$e" = "-" ]; then ee=""; else ee="$e"; fi
    env $ee timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline --no-local-map --no-host-fed \
        --steps ${STEPS:-50} --parity-frames 16 $EXTRA > gpurun_out/abenvp.json 2> gpurun_out/abenvp.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/abenvp.json')); s=d['roofline']['stage_ms']; print('$WL [$e]', d['value'], d['ms_per_step'], d['parity'].get('bit_exact'), {k: round(x, 3) for k, x in s.items()}, flush=True)" || exit 1
  done
done
