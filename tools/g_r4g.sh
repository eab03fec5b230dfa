# Fused FAST NMS: extraction parity, then pipelined A/B against HEAD's library.
set -o pipefail
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_gpu_extract.py tests/test_gpu_extract_edges.py tests/test_gpu_pipeline.py tests/test_gpu_keyframes.py > gpurun_out/r4g_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r4g_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib.sh 2 tum head base && bash tools/ab_lib.sh 1 tum5k head base
