# Replay without non-blocking sequence points: matcher parity, then the drop-in rows.
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_posed.py tests/test_gpu_pipeline.py > gpurun_out/r04q_pytest.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --rows --reps 20 > gpurun_out/r04q_rows.json 2> gpurun_out/r04q_rows.err || exit 2
ORBX_CALL_STAMPS=1 timeout -k 10 400 python bench.py --rows --reps 5 > gpurun_out/r04q_rows_st.json 2> gpurun_out/r04q_rows_st.err || exit 3
echo ok
