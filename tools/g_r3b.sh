set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err || exit 1
bash tools/prof_bench.sh r03a tum || exit 1
bash tools/prof_bench.sh r03a tum5k || exit 1
echo done
