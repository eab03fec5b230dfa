# Round 4, first pass: every GPU test (incl. the one-rank RCCL keyframe test and the
# bench-shape cases), the driver's default bench line, the EuRoC bench through the RCCL
# exchange, and VALU passes of configs[1] / configs[4] at HEAD.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r04a_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r04a_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || exit 3
echo bench ok
timeout -k 10 300 python bench.py --workload euroc --collective > gpurun_out/r04a_euroc_bench.json 2> gpurun_out/r04a_euroc_bench.err || exit 4
echo euroc ok
bash tools/pmc_valu.sh r04a tum || exit 5
bash tools/pmc_valu.sh r04a tum5k || exit 6
echo done
