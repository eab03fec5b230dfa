# HBM traffic per kernel launch (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE
# in separate rocprofv3 --pmc passes (counters only, no traces), then summarised into
# profiles/<TAG>_pmc_traffic.json by tools/pmc_traffic.py.
# usage: bash tools/pmc_traffic.sh TAG [SCRIPT]   (SCRIPT: bench.py by default, or "bench.py --vocab" / "bench.py --rows")
set -o pipefail
TAG=${1:-run}
R=$(pwd)
SCRIPT=${2:-bench.py}
EXTRA=""
[ "$SCRIPT" = "bench.py --vocab" ] && EXTRA="--parity-frames 0"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_fetch -o run -- python $R/$SCRIPT --steps 2 --warmup 1 --no-cpu-baseline $EXTRA > $R/gpurun_out/${TAG}_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_write -o run -- python $R/$SCRIPT --steps 2 --warmup 1 --no-cpu-baseline $EXTRA > $R/gpurun_out/${TAG}_write.log 2>&1
rc=$?
echo "pmc_traffic rc=$rc"
exit $rc
