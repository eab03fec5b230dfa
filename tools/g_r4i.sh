# Full GPU suite at the working tree, then the driver-shaped bench (only the dominant
# stage's events in the timed loop) A/B against HEAD's library (every stage's events).
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4i_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4i_pytest.log; [ $rc -ne 0 ] && exit $rc
STEPS=20 EXTRA="--warmup 5" bash tools/ab_lib.sh 3 tum head base
