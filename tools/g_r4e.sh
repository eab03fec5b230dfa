# Tile-major describe: parity (auto: tiles at configs[4]; forced on everywhere), then A/B.
set -o pipefail
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests/test_gpu_extract.py tests/test_gpu_extract_edges.py tests/test_gpu_pipeline.py > gpurun_out/r4e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4e_pytest.log; [ $rc -ne 0 ] && exit $rc
ORBX_DESC_TILES=1 timeout -k 10 400 $T tests/test_gpu_extract.py tests/test_gpu_extract_edges.py tests/test_gpu_pipeline.py > gpurun_out/r4e_pytest_forced.log 2>&1
rc=$?; tail -3 gpurun_out/r4e_pytest_forced.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_envp.sh 2 tum5k - ORBX_DESC_TILES=0 && bash tools/ab_envp.sh 2 tum - ORBX_DESC_TILES=1
