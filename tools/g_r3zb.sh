# Matcher stream priority beside the extraction (ORBX_MATCH_STREAM_PRIO), variants a / b.
set -o pipefail
mkdir -p gpurun_out
for w in tum5k tum; do
  for pr in 0 -1; do
    for v in ${VARIANTS:-a b}; do
      ORBX_MATCH_STREAM_PRIO=$pr ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --workload $w \
          --no-cpu-baseline --no-local-map --no-host-fed --steps 30 --parity-frames 16 > gpurun_out/r3zb.json 2>gpurun_out/r3zb.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3zb.json')); s=d['roofline']['stage_ms']; print('$w prio $pr $v', d['value'], d['ms_per_step'], d['parity']['bit_exact'], round(s['describe'],3), round(s['match'],3), flush=True)" || exit 1
    done
  done
done
