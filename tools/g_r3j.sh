# Replay width: parity at 64 / 256 / 1024 replay threads, then the pipelined A/B and the
# drop-in host calls.
set -o pipefail
mkdir -p gpurun_out
for rt in 64 1024 256; do
  ORBX_REPLAY_THREADS=$rt timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_pipeline.py \
      tests/test_gpu_posed.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3j_pytest_$rt.log 2>&1
  rc=$?; echo "rt=$rt"; tail -2 gpurun_out/r3j_pytest_$rt.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for w in tum5k tum; do
  for i in 1 2; do
    for rt in 64 256 1024; do
      ORBX_REPLAY_THREADS=$rt timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-local-map --steps 30 \
          --parity-frames 64 > gpurun_out/r3j.json 2>gpurun_out/r3j.err || exit 1
      python3 -c "import json; d=json.load(open('gpurun_out/r3j.json')); print('$w rt=$rt', d['value'], d['ms_per_step'], d['parity']['bit_exact'], {k: round(x,4) for k,x in d['roofline']['stage_ms'].items()}, flush=True)"
    done
  done
done
timeout -k 10 300 python bench.py --rows --reps 20 > gpurun_out/r3j_rows.json 2> gpurun_out/r3j_rows.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/r3j_rows.json'))
for r in d['rows']: print(r['row'], r['size'][:24], r['gpu_ms'], r['cpu_ms'], r['speedup'], r['bit_exact'])"
