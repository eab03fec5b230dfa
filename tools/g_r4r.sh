# Claim words (blocking flag in LDS): full GPU suite, then the drop-in rows with call stamps.
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r04r_pytest.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --rows --reps 20 > gpurun_out/r04r_rows.json 2> gpurun_out/r04r_rows.err || exit 2
ORBX_CALL_STAMPS=1 timeout -k 10 400 python bench.py --rows --reps 5 > gpurun_out/r04r_rows_st.json 2> gpurun_out/r04r_rows_st.err || exit 3
echo ok
