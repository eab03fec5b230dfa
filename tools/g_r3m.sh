# Matcher parity, then phases of the drop-in projection calls (ORBX_CALL_STAMPS) at replay
# width 64 / 256 and the row bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_pipeline.py tests/test_gpu_posed.py \
    tests/test_gpu_fuse.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3m_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3m_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rt in 64 256; do
ORBX_CALL_STAMPS=1 ORBX_REPLAY_THREADS=$rt timeout -k 10 300 python bench.py --rows --reps 10 > gpurun_out/r3m_rows_$rt.json 2> gpurun_out/r3m_rows_$rt.err || exit 1
echo "rt=$rt"; grep "orbx call" gpurun_out/r3m_rows_$rt.err | awk 'NR%11==5' | head -8
ORBX_REPLAY_THREADS=$rt timeout -k 10 300 python bench.py --rows --reps 30 > gpurun_out/r3m_rowsb_$rt.json 2> gpurun_out/r3m_rowsb.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/r3m_rowsb_$rt.json'))
for r in d['rows'][3:7]: print(r['row'], r['gpu_ms'], r.get('lib_ms'), r['cpu_ms'], r['speedup'], r.get('speedup_lib'), r['bit_exact'])"
done
