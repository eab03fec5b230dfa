# A/B of library builds in the pipelined bench (the driver's step shape), interleaved.
# usage: bash tools/ab_lib.sh ROUNDS WORKLOAD TAG1 TAG2 ...
#   TAG "base" = the in-tree liborbx.so, otherwise orbslam2commentedbyxcm_amd/_ab/liborbx_TAG.so
#   (python -m orbslam2commentedbyxcm_amd.build --variant TAG -DNAME=V ...); STEPS (default 50) and
#   EXTRA (more bench.py args) from the environment.
set -o pipefail
N=$1; WL=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in "$@"; do
    if [ "$v" = "base" ]; then lib=""; else lib="ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so"; fi
    env $lib timeout -k 10 200 python bench.py --workload $WL --no-cpu-baseline --no-local-map --no-host-fed \
        --steps ${STEPS:-50} --parity-frames 16 $EXTRA > gpurun_out/ablib_$v.json 2> gpurun_out/ablib_$v.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ablib_$v.json')); s=d['roofline']['stage_ms']; print('$WL $v', d['value'], d['ms_per_step'], d['parity'].get('bit_exact'), {k: round(x, 3) for k, x in s.items()}, flush=True)" || exit 1
  done
done
