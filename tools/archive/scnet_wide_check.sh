#!/bin/bash
# SCNet wide-width parity (large / intermediate dims) + same-box A/B of the LSTM recurrence kernel
# choice for H 160..256 (SESA_LSTM_WIDE_MIN_NW=9: streamed register kernel; =5: wide ring kernel).
set -e
O=gpurun_out/scw
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[scw] $(date +%T) tests"
timeout -k 10 400 python -u -m pytest tests/test_scnet.py -m gpu -x -v --timeout 150 --timeout-method thread -s > $O/test.log 2>&1
echo "[scw] $(date +%T) bench A (min_nw 9)"
SESA_LSTM_WIDE_MIN_NW=9 timeout -k 10 300 python bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_A.json 2> $O/bench_A.err
echo "[scw] $(date +%T) bench B (min_nw 5)"
SESA_LSTM_WIDE_MIN_NW=5 timeout -k 10 300 python bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_B.json 2> $O/bench_B.err
echo "[scw] $(date +%T) bench A2"
SESA_LSTM_WIDE_MIN_NW=9 timeout -k 10 300 python bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_A2.json 2> $O/bench_A2.err
echo "[scw] $(date +%T) done"
