# A full GPU pass: every -m gpu test, the default bench line, its kernel-trace profile,
# and the HBM-traffic (FETCH_SIZE, WRITE_SIZE) and VALU-issue PMC passes.  Each GPU step
# has its own time limit; any failure ends the script.
# usage: bash tools/gpu_full.sh TAG     (then: python tools/pmc_traffic.py TAG; python tools/pmc_valu.py TAG)
set -o pipefail
TAG=${1:-full}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o run -- \
    python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --parity-frames 0 > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_fetch -o run -- \
    python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-frames 0 > $R/gpurun_out/${TAG}_fetch.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_write -o run -- \
    python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-frames 0 > $R/gpurun_out/${TAG}_write.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $R/gpurun_out/${TAG}_valu -o run -- \
    python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --parity-frames 0 > $R/gpurun_out/${TAG}_valu.log 2>&1 || exit 1
echo "gpu_full ok"
