#!/bin/bash
# Round 5 lease AD: execution-batch A/B on the final tree -- MDX23C 57 (3 forwards) vs 85 (2), HTDemucs 48 (14) vs 64 (11).
set -e
O=gpurun_out/r05ad
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[r05ad] $(date +%T) $*"; }
for eb in 57 85 57; do
  step mdx23c eb $eb
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-pcie --exec-batch $eb > $O/mdx_$eb.json 2> $O/mdx_$eb.err
  python3 -c "import json; d=json.load(open('$O/mdx_$eb.json')); print('mdx23c', $eb, d['value'], d['ms_per_step'])"
done
for eb in 48 64 48; do
  step htdemucs eb $eb
  timeout -k 10 300 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-pcie --exec-batch $eb > $O/htd_$eb.json 2> $O/htd_$eb.err
  python3 -c "import json; d=json.load(open('$O/htd_$eb.json')); print('htdemucs', $eb, d['value'], d['ms_per_step'])"
done
step done
