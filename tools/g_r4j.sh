# k_describe8 (eight keypoints per wave): parity with ORBX_DESC_KPW=8, then pipelined A/B.
set -o pipefail
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
ORBX_DESC_KPW=8 timeout -k 10 400 $T tests/test_gpu_extract.py tests/test_gpu_extract_edges.py tests/test_gpu_pipeline.py -k "not local_map" > gpurun_out/r4j_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4j_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_envp.sh 2 tum - ORBX_DESC_KPW=8 && bash tools/ab_envp.sh 2 tum5k - ORBX_DESC_KPW=8
