# Drop-in host calls: the row bench and its kernel / copy trace.
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)

cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3i_prof -o run -- \
    python3 $R/bench.py --rows --reps 20 > $R/gpurun_out/r3i_prof.log 2>&1 || exit 1
echo done
