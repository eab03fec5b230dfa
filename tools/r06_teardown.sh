# Round 6: the exit-time teardown and every-rank / every-frame parity, one pass each.
#   1. the configs[3] --collective command that died at exit under rocprofv3 in r05e, once
#      without and once under rocprofv3 --kernel-trace (exit status and stderr recorded);
#   2. the world-2 one-GPU rehearsal of the N-GPU headline (gloo, both ranks on GPU 0):
#      parity.ranks_checked must be 2;
#   3. the C++ drop-in threads with every frame compared.
set -o pipefail
TAG=${1:-r06c}
R=$(pwd)
mkdir -p gpurun_out
CMD="python3 $R/bench.py --workload euroc --no-cpu-baseline --parity-frames 0 --collective"
timeout -k 10 300 $CMD > gpurun_out/${TAG}_collective.json 2> gpurun_out/${TAG}_collective.err
echo "collective (no profiler) exit $?"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/${TAG}_collective_prof -o run -- $CMD > $R/gpurun_out/${TAG}_collective_prof.json \
    2> $R/gpurun_out/${TAG}_collective_prof.err )
echo "collective (rocprofv3) exit $?"
grep -c "SIGSEGV\|Fatal Python\|Aborted" gpurun_out/${TAG}_collective.err gpurun_out/${TAG}_collective_prof.err
ORBX_BENCH_SHARE_GPU=1 ORBX_BENCH_PG=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 3 \
    --no-cpu-baseline > gpurun_out/${TAG}_world2.json 2> gpurun_out/${TAG}_world2.err || { tail -20 gpurun_out/${TAG}_world2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_world2.json').read().splitlines()[-1]); p=d['parity']; print('world2', d['value'], p['bit_exact'], p['ranks_checked'], p['frames_checked_all_ranks'], p['pairs_checked_all_ranks'], d['keyframe_exchange']['parity'] if d.get('keyframe_exchange') else None)"
timeout -k 10 300 python3 bench.py --dropin --cpp --threads 1,4,8 --seconds 2 > gpurun_out/${TAG}_dropin_cpp.json \
    2> gpurun_out/${TAG}_dropin_cpp.err || { tail -20 gpurun_out/${TAG}_dropin_cpp.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_dropin_cpp.json').read().splitlines()[-1]); print('dropin', d['all_bit_exact'], d['frames_run'], d['frames_checked'], d['frames_mismatched'], [r['frames_per_s'] for r in d['rows']])"
