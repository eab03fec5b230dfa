# configs[4] with the deep-pyramid lane offset (after the octree): pipeline parity tests,
# the kernel trace + PMC traffic of the driver's command (collected into profiles/ on the
# box as well, so the line reads them), then the configs[4] and configs[1] bench lines.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03s}
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -5 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
bash tools/prof_bench.sh $T tum5k || exit 1
python3 tools/prof_collect.py $T tum5k || exit 1
timeout -k 10 400 python3 bench.py --workload tum5k > gpurun_out/${T}_tum5k_bench.json 2> gpurun_out/${T}_tum5k_bench.err || exit 1
echo tum5k ok
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
echo bench ok
