# Global (not flat) loads in the matcher and the pyramid: GPU suite, rows with call stamps,
# sequence stamps, then the four bench workloads.
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r04t_pytest.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --rows --reps 20 > gpurun_out/r04t_rows.json 2> gpurun_out/r04t_rows.err || exit 2
ORBX_CALL_STAMPS=1 timeout -k 10 400 python bench.py --rows --reps 3 > gpurun_out/r04t_rows_st.json 2> gpurun_out/r04t_rows_st.err || exit 3
for w in tum tum5k; do
ORBX_MATCH_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/r04t_st_$w.json 2> gpurun_out/r04t_st_$w.err || exit 4
done
for w in tum tum5k kitti euroc; do
timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04t_bench_$w.json 2> gpurun_out/r04t_bench_$w.err || exit 5
done
echo ok
