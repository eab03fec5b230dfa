# Check of the built tree: every GPU test, smoke(), and the bench lines of configs[1] and
# configs[4].
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r3x}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${T}_smoke.log
for w in tum tum5k; do
  timeout -k 10 400 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/${T}_${w}.json 2> gpurun_out/${T}_${w}.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_${w}.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['parity']['bit_exact'], d.get('with_local_map',{}).get('value'), d.get('host_fed',{}).get('value'))"
done
