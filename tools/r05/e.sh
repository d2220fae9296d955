#!/bin/bash
# Round 5 lease E: the GPU suite on the tree (MDMA default, HTDemucs DConv apply / Gram rewrite, ensemble gate over
# three fixtures x seven methods), then benches: HTDemucs (A/B of the DConv apply), ensemble (blend parity), MDX23C.
set -e
O=gpurun_out/r05e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05e] $(date +%T) gpu suite"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s > $O/gputest.txt 2>&1 || rc=$?
tail -3 $O/gputest.txt
if [ "${rc:-0}" != 0 ]; then echo "[r05e] gpu suite rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
echo "[r05e] $(date +%T) bench htdemucs"
timeout -k 10 300 python bench.py --model htdemucs --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_htd.json 2> $O/bench_htd.err
echo "[r05e] $(date +%T) bench htdemucs (round-4 DConv apply)"
SESA_HTD_DCAPPLY=0 timeout -k 10 300 python bench.py --model htdemucs --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_htd_old.json 2> $O/bench_htd_old.err
echo "[r05e] $(date +%T) bench ensemble"
timeout -k 10 400 python bench.py --model ensemble --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_ens.json 2> $O/bench_ens.err
echo "[r05e] $(date +%T) bench mdx23c"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_mdx.json 2> $O/bench_mdx.err
echo "[r05e] $(date +%T) done"
