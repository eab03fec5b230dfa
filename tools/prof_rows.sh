# Kernel trace of the drop-in single calls (bench.py --rows, selected rows): every launch
# of every call, for the per-call breakdowns in profiles/<TAG>_rows_call_trace.txt
# (python tools/rows_trace.py TAG).
# usage: bash tools/prof_rows.sh TAG [ROWS]     (ROWS: comma-separated row ids, default a2)
set -o pipefail
TAG=${1:?tag}
ROWS=${2:-a2}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_rows_prof -o run -- \
    python3 $R/bench.py --rows --only $ROWS --reps 30 > $R/gpurun_out/${TAG}_rows_prof.json 2> $R/gpurun_out/${TAG}_rows_prof.err \
    || { tail -5 $R/gpurun_out/${TAG}_rows_prof.err; exit 1; }
echo "prof_rows ok"
