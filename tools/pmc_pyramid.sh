# Compute-side PMC counters of the extraction kernels for one library build.
# usage: bash tools/pmc_pyramid.sh TAG [LIB]
set -o pipefail
TAG=${1:-run}
R=$(pwd)
if [ -n "$2" ]; then export ORBX_LIB=$R/$2; fi
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/${TAG}_p1 -o run -- python $R/tools/prof_driver.py --steps 2 > $R/gpurun_out/${TAG}_p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_p2 -o run -- python $R/tools/prof_driver.py --steps 2 > $R/gpurun_out/${TAG}_p2.log 2>&1
rc=$?
echo "pmc_pyramid rc=$rc"
exit $rc
