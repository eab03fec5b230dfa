# The world-2 one-GPU rehearsal (gloo, both ranks on GPU 0) of the configs[4] RGB-D bench:
# every rank checks its own last batch (parity.ranks_checked must be 2).
set -o pipefail
TAG=${1:-r06}
mkdir -p gpurun_out
ORBX_BENCH_SHARE_GPU=1 ORBX_BENCH_PG=gloo timeout -k 10 400 python3 bench.py --workload tum5k --gpus 2 --steps 10 \
    --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_tum5k_world2.json 2> gpurun_out/${TAG}_tum5k_world2.err \
    || { tail -20 gpurun_out/${TAG}_tum5k_world2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_tum5k_world2.json').read().splitlines()[-1]); p=d['parity']; print('tum5k world2', d['value'], p['bit_exact'], p['ranks_checked'], p.get('frames_checked_all_ranks'), p.get('pairs_checked_all_ranks'))"
