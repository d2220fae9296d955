#!/bin/bash
# Round 5 lease B: workspace hygiene of every native forward (tools/ws_guard.py) + configs[4] blend parity scan.
set -e
O=gpurun_out/r05b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05b] $(date +%T) ws_guard"
timeout -k 10 400 python -u tools/ws_guard.py > $O/ws_guard.txt 2>&1
echo "[r05b] $(date +%T) ens scan"
timeout -k 10 400 python -u tools/ens_parity_scan.py > $O/ens_scan.txt 2>&1
echo "[r05b] $(date +%T) done"
