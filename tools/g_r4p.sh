# Drop-in rows at HEAD (in-library call clock vs one CPU core), plus a11/a12 call phase stamps.
set -o pipefail
timeout -k 10 400 python bench.py --rows --reps 20 > gpurun_out/r04p_rows.json 2> gpurun_out/r04p_rows.err || exit 1
ORBX_CALL_STAMPS=1 timeout -k 10 400 python bench.py --rows --reps 5 > gpurun_out/r04p_rows_st.json 2> gpurun_out/r04p_rows_st.err || exit 2
echo ok
