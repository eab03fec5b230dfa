# A/B timing of two library builds (orbslam2commentedbyxcm_amd/_ab/liborbx_{a,b}.so),
# alternating runs of the non-pipelined bench; prints value and stage times per run.
# usage: bash tools/ab.sh [rounds]
set -o pipefail
N=${1:-2}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in ${VARIANTS:-a b}; do
    ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --no-pipeline --no-cpu-baseline --steps 30 --parity-frames 0 > gpurun_out/ab_$v$i.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$v$i.json')); print('$v', d['value'], {k: round(x,4) for k,x in d['roofline']['stage_ms'].items()})"
  done
done
