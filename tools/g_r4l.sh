# Level 0 read in place: every GPU test, then pipelined A/B against the copy (ORBX_L0_COPY=1).
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4l_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4l_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_envp.sh 3 tum ORBX_L0_COPY=1 - && STEPS=30 bash tools/ab_envp.sh 2 tum5k ORBX_L0_COPY=1 -
