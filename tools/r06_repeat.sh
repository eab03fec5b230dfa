# Run-to-run spread of the driver's commands on one box: N runs of bench.py --steps 20 --warmup 5
# per workload (each its own process), values printed one per line.
set -o pipefail
N=${1:-8}; shift
mkdir -p gpurun_out
for wl in "$@"; do
  for i in $(seq 1 $N); do
    timeout -k 10 300 python3 bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --parity-frames 16 \
        > gpurun_out/rep_${wl}_$i.json 2> gpurun_out/rep_${wl}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/rep_${wl}_$i.json').read().splitlines()[-1]); print('$wl', $i, d['value'], d['ms_per_step'], d['parity'].get('bit_exact'), flush=True)"
  done
done
