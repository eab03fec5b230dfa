# Unaligned input rows (KITTI): aligned dword pairs instead of byte loads in k_pyramid.
set -o pipefail
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_extract.py tests/test_gpu_extract_edges.py tests/test_gpu_match.py -k "stereo or extract or pyramid" > gpurun_out/r4o_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4o_pytest.log; [ $rc -ne 0 ] && exit $rc
EXTRA="--steps 20" bash tools/ab_lib.sh 2 kitti head base
