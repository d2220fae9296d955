#!/bin/bash
# Round 5 lease S: the fused iSTFT with the next frame's spectrum prefetched under the current frame's FFT
# (SESA_HTD_ISTFT_FUSED=1) vs the frames + overlap-add kernels: HTDemucs GPU tests with it on, same-box benches.
set -e
O=gpurun_out/r05s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05s] $(date +%T) tests (fused iSTFT)"
SESA_HTD_ISTFT_FUSED=1 timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests.txt 2>&1
b() {
  echo "[r05s] $(date +%T) bench $1"
  timeout -k 10 400 python bench.py $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
b base "--model htdemucs --steps 3 --warmup 1 --no-parity"
SESA_HTD_ISTFT_FUSED=1 b fused "--model htdemucs --steps 3 --warmup 1"
b base2 "--model htdemucs --steps 3 --warmup 1 --no-parity"
SESA_HTD_ISTFT_FUSED=1 b fused2 "--model htdemucs --steps 3 --warmup 1 --no-parity"
echo "[r05s] $(date +%T) done"
