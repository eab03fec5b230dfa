# configs[1]/[4] replay stamps (lean form) and configs[4] kernel trace of the timed bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in tum tum5k; do
ORBX_MATCH_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/r04u_st_$w.json 2> gpurun_out/r04u_st_$w.err || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04u_prof_tum5k -o run -- python bench.py --workload tum5k --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04u_prof_tum5k.json 2> gpurun_out/r04u_prof_tum5k.err || exit 2
echo ok
