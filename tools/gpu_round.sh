# One GPU-box pass: parity tests, the default bench line, a kernel-trace profile of the bench.
# usage: bash tools/gpu_round.sh TAG [pytest selection]
# A test *failure* (pytest exit 1) still lets the bench run; a crash, abort, fault or
# time-out (any other non-zero status) ends the script before the next GPU step.
set -o pipefail
TAG=${1:-run}
SEL=${2:-tests}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
echo "bench rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- \
    python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --parity-frames 0 > $R/gpurun_out/${TAG}_prof.log 2>&1
rc=$?
echo "gpu_round rc=$rc"
exit $rc
