# Row-block size of the octave runs: parity with 4-row blocks, scoring stamps and A/B
# (a = 8 rows, b = 4, c = 2).
set -o pipefail
mkdir -p gpurun_out
for v in b c; do
ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py \
    tests/test_gpu_pipeline.py tests/test_gpu_posed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3u_pytest_$v.log 2>&1
rc=$?; echo "parity $v"; tail -1 gpurun_out/r3u_pytest_$v.log
if [ $rc -ne 0 ]; then exit $rc; fi
done
VARIANTS="a b c" bash -c '
for w in tum5k tum; do
  for v in $VARIANTS; do
    ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so ORBX_MATCH_STAMPS=1 ORBX_MATCH_MODE=4 timeout -k 10 150 \
        python bench.py --workload $w --no-pipeline --no-cpu-baseline --no-local-map --no-host-fed --parity-frames 0 --steps 3 --warmup 1 \
        > gpurun_out/r3u_st.json 2> gpurun_out/r3u_st_$w$v.err || exit 1
    echo "$w $v"; grep stamps gpurun_out/r3u_st_$w$v.err | tail -1 | cut -c1-150
  done
done
for w in tum5k tum; do
  for i in 1 2; do
    for v in $VARIANTS; do
      ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 200 python bench.py --workload $w \
          --no-cpu-baseline --no-local-map --no-host-fed --steps 30 --parity-frames 64 > gpurun_out/r3u.json 2>gpurun_out/r3u.err || exit 1
      python3 -c "import json; d=json.load(open(\"gpurun_out/r3u.json\")); print(\"$w $v\", d[\"value\"], d[\"ms_per_step\"], d[\"parity\"][\"bit_exact\"], round(d[\"roofline\"][\"stage_ms\"][\"match\"],4), flush=True)"
    done
  done
done'
