# PMC + kernel-trace passes over one short bench run:  bash tools/pmc_model.sh MODEL TAG KERNEL [SECONDS]
# (one --pmc pass per counter group, within the per-block slot limits; results under gpurun_out/)
set -e
M=$1; TAG=$2; K=$3; S=${4:-24}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --model $M --steps 1 --warmup 0 --track-seconds $S --no-cpu-baseline"
O=gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $O/pmc_${TAG}_sq -o run -- $B > $O/pmc_${TAG}_sq.json 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${TAG}_f -o run -- $B > /dev/null 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${TAG}_w -o run -- $B > /dev/null 2>&1
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pmc_${TAG}_h -o run -- $B > /dev/null 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof_${TAG} -o run -- $B > $O/prof_${TAG}.json 2>&1
python3 tools/pmc_sq.py $O/pmc_${TAG}_sq $O/pmc_${TAG}_h > $O/pmc_${TAG}_sq.txt
python3 tools/pmc_traffic.py $O/pmc_${TAG}_f $O/pmc_${TAG}_w "$K" $O/pmc_${TAG}_traffic.json
python3 tools/rocprof_summary.py $O/prof_${TAG} $O/prof_${TAG}_summary.txt
