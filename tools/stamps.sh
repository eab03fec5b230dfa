# Matcher phase stamps (k_proj_search, --no-pipeline) at C5 and C1.
set -o pipefail
mkdir -p gpurun_out
for w in tum5k tum; do
  ORBX_MATCH_STAMPS=1 timeout -k 10 150 python bench.py --workload $w --no-pipeline --no-cpu-baseline --parity-frames 0 --steps 3 --warmup 1 > gpurun_out/st_$w.json 2> gpurun_out/st_$w.err || exit 1
  echo $w; grep stamps gpurun_out/st_$w.err | tail -1
done
