# Kernel trace of the drop-in host calls (row bench).
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3q_prof -o run -- \
    python3 $R/bench.py --rows --reps 30 > $R/gpurun_out/r3q_prof.log 2>&1 || exit 1
echo done
