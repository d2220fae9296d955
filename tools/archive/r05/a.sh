#!/bin/bash
# Round 5 lease A: streams=2 diagnostic (tools/streams_debug3.py) + a baseline MDX23C bench line.
set -e
O=gpurun_out/r05a
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05a] $(date +%T) streams diagnostic"
timeout -k 10 300 python -u tools/streams_debug3.py 3 > $O/streams3.txt 2>&1
echo "[r05a] $(date +%T) bench"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_mdx.json 2> $O/bench_mdx.err
echo "[r05a] $(date +%T) done"
