# Row bench (per-call drop-in latency) for variants a / b.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for v in ${VARIANTS:-a b}; do
  ORBX_LIB=$PWD/orbslam2commentedbyxcm_amd/_ab/liborbx_$v.so timeout -k 10 300 python bench.py --rows > gpurun_out/r3zd_rows_$v.json 2> gpurun_out/r3zd_rows_$v.err || exit 1
  python3 -c "
import json
d=json.load(open('gpurun_out/r3zd_rows_$v.json'))
print('$v', ' '.join('%s:%s' % (r['row'], r.get('lib_ms')) for r in d['rows'] if r['row'] in ('a11','a12','a13','a14','a15','f2')))
" || exit 1
done
done
