# Kernel trace of the drop-in host calls (row bench), replay width 64 and 256.
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for rt in 64 256; do
ORBX_REPLAY_THREADS=$rt timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3l_prof_$rt -o run -- \
    python3 $R/bench.py --rows --reps 30 > $R/gpurun_out/r3l_prof_$rt.log 2>&1 || exit 1
done
echo done
