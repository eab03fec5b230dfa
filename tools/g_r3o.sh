# k_level_tiles ablations (timing only; outputs differ): a = shipped, s = no strength pass,
# r = no blur rows, p = no compass test (and so no strength); extraction alone, one lane.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in a s r p; do
    ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --no-match --lanes 1 \
        --no-cpu-baseline --parity-frames 0 --steps 30 > gpurun_out/r3o.json 2>gpurun_out/r3o.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3o.json')); print('$v', d['value'], {k: round(x,4) for k,x in d['roofline']['stage_ms'].items()}, flush=True)"
  done
done
