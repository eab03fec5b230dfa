# Bench lines of the four workloads (default arguments, the driver's command) against the
# committed profiles.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03f}
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
echo bench ok
for w in tum5k kitti euroc; do
  timeout -k 10 400 python3 bench.py --workload $w > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || exit 1
  echo $w ok
done
