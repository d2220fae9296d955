#!/bin/bash
# Round 5 lease M: htd_rw3_kernel with the LDS-staged 16-B epilogue stores vs the token / implicit GEMMs
# (SESA_HTD_RW3=0); the channel-pair DConv apply at h <= 8 (SESA_HTD_DCAPPLY8=1): GPU parity tests, same-box
# benches, per-shape conv times, kernel-trace summary.
set -e
O=gpurun_out/r05m
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05m] $(date +%T) tests"
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.txt 2>&1
b() {
  echo "[r05m] $(date +%T) bench $1"
  timeout -k 10 400 python bench.py $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
b rw3 "--model htdemucs --steps 3 --warmup 1"
SESA_HTD_RW3=0 b gemm "--model htdemucs --steps 3 --warmup 1 --no-parity"
SESA_HTD_DCAPPLY8=1 b apq8 "--model htdemucs --steps 3 --warmup 1"
b rw3b "--model htdemucs --steps 3 --warmup 1 --no-parity"
echo "[r05m] $(date +%T) rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_htd -o htd -- python bench.py --model htdemucs --steps 1 \
  --warmup 1 --no-cpu-baseline --no-parity > $O/prof_htd.log 2>&1
echo "[r05m] $(date +%T) conv shape trace"
SESA_HTD_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python bench.py \
  --model htdemucs --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $O/trace.log 2> $O/trace_shapes.txt
echo "[r05m] $(date +%T) done"
