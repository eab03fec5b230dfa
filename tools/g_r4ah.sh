# 16-byte LDS-DMA describe staging above 3000 slots (in-tree) vs register staging (reg):
# extraction + pipeline parity, then interleaved configs[4] A/B and a configs[1] check.
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_extract.py tests/test_gpu_pipeline.py tests/test_gpu_match.py > gpurun_out/r04ah_pytest.log 2>&1 || exit 1
STEPS=20 bash tools/ab_lib.sh 3 tum5k base reg || exit 2
STEPS=20 bash tools/ab_lib.sh 1 tum base reg || exit 3
echo ok
