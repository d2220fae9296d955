#!/bin/bash
# Round 5 lease I: SCNet feature-conversion DFTs on MFMA (scn_dft_mfma_kernel) and the HTDemucs whole-row DConv layer
# (htd_dc_row_kernel): GPU parity tests of both models (+ the ensemble), same-box A/B benches (SESA_SCN_DFT=0,
# SESA_HTD_DCROW=0 restore the previous kernels) and kernel-trace summaries.
set -e
O=gpurun_out/r05i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05i] $(date +%T) tests"
timeout -k 10 900 python -u -m pytest tests/test_scnet.py tests/test_htdemucs.py tests/test_ensemble_models.py -m gpu -x \
  -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
b() {
  echo "[r05i] $(date +%T) bench $1"
  timeout -k 10 400 python bench.py $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
b scn_dft "--model scnet --steps 3 --warmup 1"
SESA_SCN_DFT=0 b scn_valu "--model scnet --steps 3 --warmup 1 --no-parity"
b htd_row "--model htdemucs --steps 3 --warmup 1"
SESA_HTD_DCROW=0 b htd_split "--model htdemucs --steps 3 --warmup 1 --no-parity"
echo "[r05i] $(date +%T) rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_scn -o scn -- python bench.py --model scnet --steps 2 \
  --warmup 1 --no-cpu-baseline --no-parity > $O/prof_scn.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_htd -o htd -- python bench.py --model htdemucs --steps 1 \
  --warmup 1 --no-cpu-baseline --no-parity > $O/prof_htd.log 2>&1
echo "[r05i] $(date +%T) done"
