#!/bin/bash
# Round 5 lease J: HTDemucs whole-row DConv, occupancy form (htd_dc_row2_kernel) vs the first row kernel
# (SESA_HTD_DCROW=1) and the split form (=0); register-resident LayerNorm / quad item statistics vs the scalar
# kernels (SESA_HTD_LNV=0 SESA_HTD_STATS4=0): GPU parity tests, same-box benches, kernel-trace summary, conv shapes.
set -e
O=gpurun_out/r05j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05j] $(date +%T) tests"
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.txt 2>&1
b() {
  echo "[r05j] $(date +%T) bench $1"
  timeout -k 10 400 python bench.py $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
b row2 "--model htdemucs --steps 3 --warmup 1"
SESA_HTD_DCROW=1 b row1 "--model htdemucs --steps 3 --warmup 1 --no-parity"
SESA_HTD_DCROW=0 b split "--model htdemucs --steps 3 --warmup 1 --no-parity"
SESA_HTD_LNV=0 SESA_HTD_STATS4=0 b row2_oldnorm "--model htdemucs --steps 3 --warmup 1 --no-parity"
b row2b "--model htdemucs --steps 3 --warmup 1 --no-parity"
echo "[r05j] $(date +%T) rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_htd -o htd -- python bench.py --model htdemucs --steps 1 \
  --warmup 1 --no-cpu-baseline --no-parity > $O/prof_htd.log 2>&1
echo "[r05j] $(date +%T) conv shape trace"
SESA_HTD_TRACE=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python bench.py \
  --model htdemucs --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $O/trace.log 2> $O/trace_shapes.txt
echo "[r05j] $(date +%T) done"
