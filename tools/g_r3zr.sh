# Drop-in call phases (ORBX_CALL_STAMPS=1, diagnostics: stamps add an allocation per
# call), then kernel traces + PMC traffic of all four workloads at HEAD (tools/prof_bench.sh).
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03o}
ORBX_CALL_STAMPS=1 timeout -k 10 300 python bench.py --rows --reps 5 > gpurun_out/${T}_stamps_rows.json 2> gpurun_out/${T}_stamps.err || exit 1
echo stamps ok
for w in tum tum5k kitti euroc; do
  bash tools/prof_bench.sh $T $w || exit 1
done
