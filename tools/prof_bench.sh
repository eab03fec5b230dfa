# The profiles a bench line's roofline reads back (bench.py profile_fields), for one
# workload: a rocprofv3 kernel trace of the exact command the driver runs (1 GPU, 20 timed
# steps, 5 warmup) and the FETCH_SIZE / WRITE_SIZE PMC passes, each in its own run.
# usage: bash tools/prof_bench.sh TAG WORKLOAD     (WORKLOAD: tum | tum5k | kitti | euroc)
# then:  python tools/prof_collect.py TAG WORKLOAD  (copies the summaries into profiles/)
set -o pipefail
TAG=${1:?tag}
WL=${2:-tum}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${WL}_prof -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --workload $WL --no-cpu-baseline --parity-frames 0 \
    > $R/gpurun_out/${TAG}_${WL}_prof.json 2> $R/gpurun_out/${TAG}_${WL}_prof.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_${WL}_fetch -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --workload $WL --no-cpu-baseline --parity-frames 0 \
    > $R/gpurun_out/${TAG}_${WL}_fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_${WL}_write -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --workload $WL --no-cpu-baseline --parity-frames 0 \
    > $R/gpurun_out/${TAG}_${WL}_write.log 2>&1 || exit 1
echo "prof_bench $WL ok"
