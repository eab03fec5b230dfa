set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_posed.py tests/test_gpu_pipeline.py -m gpu -v --timeout 300 --timeout-method thread -k "local or match_sequence or create_mappoints" > gpurun_out/r3c_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r3c_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/g_r3b.sh
