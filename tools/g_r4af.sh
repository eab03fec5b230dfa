# One-sided paired FAST strength (ORBX_LT_SIDED=1, in-tree) vs the two-sided form (sd0):
# extraction parity first, then interleaved pipelined A/B on configs[1], [4], [2].
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_pipeline.py > gpurun_out/r04af_pytest.log 2>&1 || exit 1
STEPS=20 bash tools/ab_lib.sh 3 tum base sd0 || exit 2
STEPS=20 bash tools/ab_lib.sh 2 tum5k base sd0 || exit 3
STEPS=20 bash tools/ab_lib.sh 2 kitti base sd0 || exit 4
echo ok
