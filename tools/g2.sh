set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g2_pytest.log 2>&1 || { tail -30 gpurun_out/g2_pytest.log; exit 1; }
tail -1 gpurun_out/g2_pytest.log
bash tools/stamps.sh || exit 1
for w in tum tum5k; do timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/b_$w.json 2> gpurun_out/b_$w.err || exit 1; python -c "import json; d=json.load(open('gpurun_out/b_$w.json')); print('$w', d['value'], d['ms_per_step'], d['parity']['bit_exact'], d['parity']['frames_checked'], d['parity']['pairs_checked'], d['roofline']['stage_ms'])"; done
