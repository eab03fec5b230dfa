set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_posed.py tests/test_gpu_pipeline.py tests/test_gpu_keyframes.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3a_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r3a_pytest.log
exit $rc
