# Full GPU parity after the H4 (fused) changes, smoke, and a bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3r_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3r_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r3r_bench.json 2> gpurun_out/r3r_bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r3r_bench.json')); print(d['value'], d['parity'], d['with_local_map']['value'], d['with_local_map']['parity']['bit_exact'])"
