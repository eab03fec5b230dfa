# Bench lines of all four workloads (the driver's default commands) against the newest
# committed traces, then the drop-in rows.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03p}
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
echo bench ok
for w in tum5k kitti euroc; do
  timeout -k 10 400 python3 bench.py --workload $w > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || exit 1
  echo $w ok
done
timeout -k 10 300 python bench.py --rows --reps 30 > gpurun_out/${T}_rows.json 2> gpurun_out/${T}_rows.err || exit 1
echo rows ok
