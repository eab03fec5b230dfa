# Pyramid segments (ORBX_PZ_SEG): GPU extraction parity, then configs[4] / configs[1]
# pipelined A/B (8 levels per segment, the default, against one segment), three rounds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_extract_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3zn_pytest.log 2>&1 || { tail -30 gpurun_out/r3zn_pytest.log; exit 1; }
tail -1 gpurun_out/r3zn_pytest.log
for i in 1 2 3; do
  for v in 8 0; do
    for w in tum5k; do
      ORBX_PZ_SEG=$v timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --no-host-fed \
          --steps 50 --parity-frames -1 > gpurun_out/r3zn.json 2>gpurun_out/r3zn.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3zn.json')); print('$w seg $v', d['value'], d['ms_per_step'], d['parity']['bit_exact'], d['roofline']['stage_ms']['pyramid'], flush=True)" || exit 1
    done
  done
done
