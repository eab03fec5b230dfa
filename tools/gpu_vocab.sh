# Vocabulary transform bench + kernel-trace profile on one GPU box.
# usage: bash tools/gpu_vocab.sh TAG
set -o pipefail
TAG=${1:-vocab}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --vocab > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python $R/bench.py --vocab --steps 10 --warmup 2 --no-cpu-baseline --parity-frames 0 > $R/gpurun_out/${TAG}_prof.log 2>&1
rc=$?
echo "gpu_vocab rc=$rc"
exit $rc
