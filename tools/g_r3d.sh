set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3d_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3d_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err || exit 1
echo bench ok
for w in tum5k kitti euroc; do
  timeout -k 10 300 python3 bench.py --workload $w > gpurun_out/r3d_$w.json 2> gpurun_out/r3d_$w.err || exit 1
  echo $w ok
done
bash tools/prof_bench.sh r03b kitti || exit 1
bash tools/prof_bench.sh r03b euroc || exit 1
echo done
