# k_local_build workgroups per frame: parity (local-map tests), then the with_local_map leg at configs[1] / configs[4].
set -o pipefail
mkdir -p gpurun_out
ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_b.so timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_posed.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zg_pytest.log 2>&1
rc=$?; echo "parity b"; tail -1 gpurun_out/r3zg_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in tum5k tum; do
  for i in 1 2; do
    for v in a b; do
      ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline --no-host-fed \
          --steps 20 --parity-frames 8 > gpurun_out/r3zg.json 2>gpurun_out/r3zg.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3zg.json')); print('$w $v', d['value'], d['with_local_map']['value'], d['parity']['bit_exact'], flush=True)" || exit 1
    done
  done
done
