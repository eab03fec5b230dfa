# Adaptive replay width of the single calls: matcher parity, then the row bench (with the
# per-call stamps: duplicates and the chosen replay).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_posed.py tests/test_gpu_pipeline.py tests/test_gpu_fuse.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3za_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/r3za_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
ORBX_CALL_STAMPS=1 timeout -k 10 300 python bench.py --rows > gpurun_out/r3za_rows_st.json 2> gpurun_out/r3za_rows_st.err || exit 1
timeout -k 10 300 python bench.py --rows > gpurun_out/r3za_rows.json 2> gpurun_out/r3za_rows.err || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/r3za_rows.json'))
for r in d['rows']:
    print(r['row'], r['size'][:22], r.get('lib_ms'), r['cpu_ms'], r.get('speedup_lib'), r['bit_exact'])
"
