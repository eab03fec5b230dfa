set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --no-local-map > gpurun_out/r3t.json 2> gpurun_out/r3t.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r3t.json')); print(d['value'], d['parity']['bit_exact'], d['host_fed'])"
