# One GPU-box pass: parity tests, the default bench line, a kernel-trace profile of the bench.
# usage: bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${TAG}_prof.log 2>&1
rc=$?
echo "gpu_round rc=$rc"
exit $rc
