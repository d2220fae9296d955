#!/bin/bash
# Round 4: conv3x3 fp16 shortcut phase on the per-wave LDS-DMA ring (SCR=2) vs the LDS-staged shortcut,
# per level, with the identity check.
set -e
O=gpurun_out/r04e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04e] $(date +%T) conv_bench f16"
timeout -k 10 300 ./tools/conv_bench 57 f16 > $O/conv_f16.txt 2>&1
echo "[r04e] $(date +%T) done"
