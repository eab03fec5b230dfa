set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc1 -o run -- python tools/prof_driver.py --steps 2 > gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc2 -o run -- python tools/prof_driver.py --steps 2 > gpurun_out/pmc2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc3 -o run -- python tools/prof_driver.py --steps 2 > gpurun_out/pmc3.log 2>&1
echo rc=$?
ls gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3
