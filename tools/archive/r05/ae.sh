#!/bin/bash
# Round 5 lease AE: MDX23C execution batch 57 (3 forwards) vs 43 (4 forwards, what cap 96 plans after the workspace
# guard halves it) vs 57, same box.
set -e
O=gpurun_out/r05ae
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for eb in 57 43 57; do
  echo "[r05ae] $(date +%T) mdx23c eb $eb"
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-pcie --exec-batch $eb > $O/mdx_$eb.json 2> $O/mdx_$eb.err
  python3 -c "import json; d=json.load(open('$O/mdx_$eb.json')); print('mdx23c', $eb, d['value'], d['ms_per_step'])"
done
echo "[r05ae] $(date +%T) done"
