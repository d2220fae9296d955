#!/bin/bash
# Round 5 lease H: SCNet feature-conversion DFTs on MFMA (scn_dft_mfma_kernel) -- SCNet GPU parity tests, bench
# with the MFMA DFTs and with the VALU direct DFTs (SESA_SCN_DFT=0), and a kernel-trace summary.
set -e
O=gpurun_out/r05h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05h] $(date +%T) scnet tests"
timeout -k 10 600 python -u -m pytest tests/test_scnet.py tests/test_ensemble_models.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests.txt 2>&1
echo "[r05h] $(date +%T) bench dft"
timeout -k 10 400 python bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_dft.json 2> $O/bench_dft.err
echo "[r05h] $(date +%T) bench valu"
SESA_SCN_DFT=0 timeout -k 10 400 python bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline --no-parity \
  > $O/bench_valu.json 2> $O/bench_valu.err
echo "[r05h] $(date +%T) rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o scn -- python bench.py --model scnet --steps 2 \
  --warmup 1 --no-cpu-baseline --no-parity > $O/prof.log 2>&1
echo "[r05h] $(date +%T) done"
