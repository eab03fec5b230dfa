# Fused FAST NMS vs HEAD (both with every stage's events in the timed loop), then the
# working tree with only the dominant stage's events (the bench default).
set -o pipefail
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_extract.py tests/test_gpu_pipeline.py -k "not local_map" > gpurun_out/r4h_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4h_pytest.log; [ $rc -ne 0 ] && exit $rc
ORBX_BENCH_ALL_EVENTS=1 bash tools/ab_lib.sh 2 tum head base && bash tools/ab_lib.sh 1 tum base && \
ORBX_BENCH_ALL_EVENTS=1 bash tools/ab_lib.sh 1 tum5k head base
