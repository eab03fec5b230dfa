# HBM traffic per kernel launch (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE
# in separate rocprofv3 --pmc passes (counters only, no traces), then summarised into
# profiles/<TAG>_pmc_traffic.json by tools/pmc_traffic.py.
# usage: bash tools/pmc_traffic.sh TAG
set -o pipefail
TAG=${1:-run}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_fetch -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_write -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_write.log 2>&1
rc=$?
echo "pmc_traffic rc=$rc"
exit $rc
