#!/bin/bash
# MFMA-pipe utilisation per kernel over one short bench run (one --pmc pass, its own time limit):
#   bash tools/pmc_mfma.sh MODEL TAG [SECONDS] [EXTRA bench args]
# busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (MI355X_MICROARCH.md: the MFMA
# busy counter counts cycles, GRBM_GUI_ACTIVE is summed over the 8 XCDs).
set -e
M=$1; TAG=$2; S=${3:-24}; EXTRA=${4:-}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --model $M --steps 1 --warmup 0 --track-seconds $S --no-cpu-baseline --no-parity $EXTRA"
O=gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_${TAG}_mfma -o run -- $B > $O/pmc_${TAG}_mfma.log 2>&1
python3 tools/pmc_mfma.py $O/pmc_${TAG}_mfma > $O/pmc_${TAG}_mfma.txt
rm -rf $O/pmc_${TAG}_mfma
