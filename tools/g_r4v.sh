# Replay phase breakdown (lean form, 256-thread replay) at configs[1] and configs[4].
set -o pipefail
for w in tum tum5k; do
ORBX_MATCH_STAMPS=1 timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-pipeline > gpurun_out/r04v_st_$w.json 2> gpurun_out/r04v_st_$w.err || exit 1
done
echo ok
