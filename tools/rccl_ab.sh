# configs[3] (EuRoC keyframes): what the RCCL slab all-gather adds to the step at world
# size 1 -- ROUNDS interleaved runs of the in-place step, the step with the exchange through
# the process group waited for by the matcher stream (ORBX_GATHER_SYNC=1, round 4's order)
# and the same with only the triangulation stream waiting (the default since round 5), on
# one box; then a kernel trace of the --collective run.
# usage: bash tools/rccl_ab.sh TAG [ROUNDS]   then: python tools/rccl_summary.py TAG
set -o pipefail
TAG=${1:?tag}
N=${2:-3}
R=$(pwd)
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for mode in inplace sync collective; do
    extra="--collective"
    envs=""
    [ $mode = inplace ] && extra=""
    [ $mode = sync ] && envs="ORBX_GATHER_SYNC=1"
    env $envs timeout -k 10 300 python bench.py --workload euroc --no-cpu-baseline --parity-frames 0 $extra \
        > gpurun_out/${TAG}_euroc_${mode}_$i.json 2> gpurun_out/${TAG}_euroc_${mode}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_euroc_${mode}_$i.json').read().splitlines()[-1]); print('$mode', d['value'], d['ms_per_step'], d['config'].get('slab_exchange'), flush=True)" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_rccl_prof -o run -- \
    python3 $R/bench.py --workload euroc --no-cpu-baseline --parity-frames 0 --collective \
    > $R/gpurun_out/${TAG}_rccl_prof.json 2> $R/gpurun_out/${TAG}_rccl_prof.err || exit 1
echo "rccl_ab ok"
