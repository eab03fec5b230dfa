# configs[1] pipelined A/B, interleaved, three rounds (variants a / b).
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in ${VARIANTS:-a b}; do
    ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-local-map --no-host-fed \
        --steps 50 --parity-frames 8 > gpurun_out/r3zk.json 2>gpurun_out/r3zk.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r3zk.json')); print('tum $v', d['value'], d['ms_per_step'], d['parity']['bit_exact'], flush=True)" || exit 1
  done
done
