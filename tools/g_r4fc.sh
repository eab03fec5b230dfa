# Round-4 final pass, part C: the bench lines with the r04f profiles committed in the tree.
set -o pipefail
timeout -k 10 300 python bench.py > gpurun_out/r04f_tum_bench.json 2> gpurun_out/r04f_tum_bench.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04f_tum_bench20.json 2> gpurun_out/r04f_tum_bench20.err || exit 2
for wl in tum5k kitti euroc; do
timeout -k 10 300 python bench.py --workload $wl > gpurun_out/r04f_${wl}_bench.json 2> gpurun_out/r04f_${wl}_bench.err || exit 3
done
echo part C done
