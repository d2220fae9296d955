#!/bin/bash
# Round 5 lease U: the interleaved fused shortcut (conv3x3_db_kernel<SCR = 3>) -- per-level micro-benchmark against the
# ring shortcut, then same-box MDX23C bench A/B/A (the B leg with the parity fixtures), GPU parity tests under SCI=1.
set -e
O=gpurun_out/r05u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05u] $(date +%T) conv_bench sci"
timeout -k 10 300 ./tools/conv_bench 57 sci > $O/conv_bench_sci.txt 2>&1
cat $O/conv_bench_sci.txt
echo "[r05u] $(date +%T) bench A (ring)"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_ring.json 2> $O/bench_ring.err
echo "[r05u] $(date +%T) bench B (interleaved)"
SESA_CONV_SCI=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_sci.json 2> $O/bench_sci.err
echo "[r05u] $(date +%T) bench A2 (ring)"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_ring2.json 2> $O/bench_ring2.err
echo "[r05u] $(date +%T) gpu tests (mdx23c, SCI=1)"
SESA_CONV_SCI=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/tests_sci.txt 2>&1
tail -3 $O/tests_sci.txt
echo "[r05u] $(date +%T) done"
