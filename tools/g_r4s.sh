# Sequence replay counters (split launches) at configs[1] and configs[4]; drop-in call stamps.
set -o pipefail
for w in tum tum5k; do
ORBX_MATCH_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/r04s_$w.json 2> gpurun_out/r04s_$w.err || exit 1
done
ORBX_CALL_STAMPS=1 timeout -k 10 400 python bench.py --rows --reps 3 > gpurun_out/r04s_rows_st.json 2> gpurun_out/r04s_rows_st.err || exit 2
echo ok
