# Kernel trace of the drop-in rows (launch gaps and per-kernel times of the single calls).
set -o pipefail
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r04ac_rows_prof -o run -- python3 $R/bench.py --rows --reps 5 > $R/gpurun_out/r04ac_rows.json 2> $R/gpurun_out/r04ac_rows.err || exit 1
echo ok
