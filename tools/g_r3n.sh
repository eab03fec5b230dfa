# Round-3 measurement pass: every GPU test, the bench lines of all four workloads, and the
# profiles the lines read back (kernel trace of the driver's exact command + PMC traffic).
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03c}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in tum tum5k kitti euroc; do
  bash tools/prof_bench.sh $T $w || exit 1
done
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
echo bench ok
for w in tum5k kitti euroc; do
  timeout -k 10 400 python3 bench.py --workload $w > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || exit 1
  echo $w ok
done
