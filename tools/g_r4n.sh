# Round-4 measurement pass at HEAD: kernel trace of the driver's command + PMC traffic per
# workload (tools/prof_bench.sh), VALU passes for configs[1] / [4], the default bench line.
set -o pipefail
for wl in tum tum5k kitti euroc; do bash tools/prof_bench.sh r04n $wl || exit 1; done
bash tools/pmc_valu.sh r04n tum || exit 2
bash tools/pmc_valu.sh r04n tum5k || exit 3
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04n_bench.json 2> gpurun_out/r04n_bench.err || exit 4
echo pass done
