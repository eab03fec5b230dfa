# Where the kernels' wave cycles go, under the driver's bench command (pipelined, two
# lanes; rocprofv3's dispatch counters serialise the dispatches, so each kernel is counted
# alone): two --pmc passes of at most 8 SQ counters each (MI355X_MICROARCH.md, PMC table),
# each in its own run.  Counters the device does not list (rocprofv3 -L) are dropped.
#   pass A: SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY
#           SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
#   pass B: SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
#           SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM, GRBM_GUI_ACTIVE
# usage: bash tools/pmc_stall.sh TAG [WORKLOAD]   ->  python tools/pmc_stall.py TAG
set -o pipefail
TAG=${1:-run}
WL=${2:-tum}
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/${TAG}_counters.txt 2>&1 || { echo "rocprofv3 -L failed"; exit 1; }
have() { for c in "$@"; do grep -qw "$c" $R/gpurun_out/${TAG}_counters.txt && printf '%s ' "$c"; done; }
A=$(have SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT)
B=$(have SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE)
echo "pass A: $A"
echo "pass B: $B"
CMD="python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --parity-frames 0 --no-local-map --no-host-fed --workload $WL"
timeout -s KILL 150 rocprofv3 --pmc $A --output-format csv -d $R/gpurun_out/${TAG}_stallA -o run -- $CMD \
    > $R/gpurun_out/${TAG}_stallA.log 2>&1 || { echo "stall A failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $B --output-format csv -d $R/gpurun_out/${TAG}_stallB -o run -- $CMD \
    > $R/gpurun_out/${TAG}_stallB.log 2>&1 || { echo "stall B failed"; exit 1; }
echo "pmc_stall ok"
