# Round-4 final pass, part B: kernel trace of the driver's command + PMC traffic per
# workload (tools/prof_bench.sh), VALU passes for configs[1] / [4], then the untraced
# bench lines (driver defaults, and 20 steps) for every workload.
set -o pipefail
for wl in tum tum5k kitti euroc; do bash tools/prof_bench.sh r04f $wl || exit 1; done
bash tools/pmc_valu.sh r04f tum || exit 2
bash tools/pmc_valu.sh r04f tum5k || exit 3
timeout -k 10 300 python bench.py > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04f_bench20.json 2> gpurun_out/r04f_bench20.err || exit 5
for wl in tum5k kitti euroc; do
timeout -k 10 300 python bench.py --workload $wl > gpurun_out/r04f_${wl}_bench.json 2> gpurun_out/r04f_${wl}_bench.err || exit 6
done
echo part B done
