# Wave-state breakdown (where the cycles go) over one short bench run:
#   bash tools/pmc_stall.sh MODEL TAG [SECONDS]
# SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stall) + SQ_ACTIVE_INST_ANY
# ~= SQ_WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots).
set -e
M=$1; TAG=$2; S=${3:-24}; EXTRA=${4:-}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --model $M --steps 1 --warmup 0 --track-seconds $S --no-cpu-baseline $EXTRA"
O=gpurun_out
timeout -s KILL 60 rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || true
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d $O/pmc_${TAG}_st -o run -- $B > /dev/null 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_${TAG}_sq -o run -- $B > /dev/null 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${TAG}_f -o run -- $B > /dev/null 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${TAG}_w -o run -- $B > /dev/null 2>&1
python3 tools/pmc_sq.py $O/pmc_${TAG}_st $O/pmc_${TAG}_sq > $O/pmc_${TAG}_stall.txt
