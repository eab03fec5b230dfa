# Drop-in host calls after the in-kernel staging: parity, call phases, the row bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_posed.py tests/test_gpu_fuse.py tests/test_cpp_mirror.py tests/test_abi.py \
    tests/test_gpu_bow.py tests/test_gpu_frame.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3p_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3p_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
ORBX_CALL_STAMPS=1 timeout -k 10 300 python bench.py --rows --reps 10 > gpurun_out/r3p_rows_st.json 2> gpurun_out/r3p_rows_st.err || exit 1
grep "orbx call" gpurun_out/r3p_rows_st.err | awk 'NR%11==5' | head -8
timeout -k 10 300 python bench.py --rows --reps 30 > gpurun_out/r3p_rows.json 2> gpurun_out/r3p_rows.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/r3p_rows.json'))
for r in d['rows']: print(r['row'], r['size'][:16], r['gpu_ms'], r.get('lib_ms'), r['cpu_ms'], r['speedup'], r.get('speedup_lib'), r['bit_exact'])"
