set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g1_pytest.log 2>&1 || { tail -30 gpurun_out/g1_pytest.log; exit 1; }
tail -3 gpurun_out/g1_pytest.log
ORBX_MATCH_STAMPS=1 timeout -k 10 150 python bench.py --workload tum5k --no-pipeline --no-cpu-baseline --parity-frames 0 --steps 3 --warmup 1 > gpurun_out/st5.json 2> gpurun_out/st5.err || exit 1
ORBX_MATCH_STAMPS=1 timeout -k 10 150 python bench.py --no-pipeline --no-cpu-baseline --parity-frames 0 --steps 3 --warmup 1 > gpurun_out/st1.json 2> gpurun_out/st1.err || exit 1
grep stamps gpurun_out/st5.err | tail -1; grep stamps gpurun_out/st1.err | tail -1
for w in tum tum5k; do timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit 1; python -c "import json; d=json.load(open('gpurun_out/b_$w.json')); print('$w', d['value'], d['ms_per_step'], d['parity'], d['roofline']['stage_ms'])"; done
