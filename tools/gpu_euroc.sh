# configs[3] (bench.py --workload euroc) line plus its kernel-trace profile.
# usage: bash tools/gpu_euroc.sh TAG
set -o pipefail
TAG=${1:-euroc}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload euroc > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- \
    python $R/bench.py --workload euroc --steps 10 --warmup 2 --no-cpu-baseline --parity-frames 0 > $R/gpurun_out/${TAG}_prof.log 2>&1
