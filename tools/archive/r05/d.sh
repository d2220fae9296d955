#!/bin/bash
# Round 5 lease D: stream-concurrency bisect (SESA_DEBUG_SYNC), configs[4] blend scan (vocals stems), conv3x3 MDMA
# micro-benchmark + same-box MDX23C bench A/B.
set -e
O=gpurun_out/r05d
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05d] $(date +%T) conv_bench mdma"
timeout -k 10 300 ./tools/conv_bench 57 mdma > $O/conv_bench_mdma.txt 2>&1
echo "[r05d] $(date +%T) bench A (regs)"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_regs.json 2> $O/bench_regs.err
echo "[r05d] $(date +%T) bench B (MDMA)"
SESA_CONV_MDMA=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_mdma.json 2> $O/bench_mdma.err
echo "[r05d] $(date +%T) bench A2 (regs)"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_regs2.json 2> $O/bench_regs2.err
echo "[r05d] $(date +%T) ens scan"
timeout -k 10 400 python -u tools/ens_parity_scan.py > $O/ens_scan.txt 2>&1
echo "[r05d] $(date +%T) streams bisect"
timeout -k 10 900 python -u tools/streams_bisect.py mdx23c bf16x3 > $O/streams_bisect.txt 2>&1
echo "[r05d] $(date +%T) done"
