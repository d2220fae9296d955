#!/bin/bash
# Round 5 lease Y: the frequency embedding fused into the level-0 rewrite store -- HTDemucs GPU tests, then the
# configs[3] and configs[1] bench lines under the HBM-resident `value` (pcie_inclusive beside it).
set -e
O=gpurun_out/r05y
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[r05y] $(date +%T) $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
step bench htdemucs
timeout -k 10 400 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_htdemucs.json 2> $O/bench_htdemucs.err
step bench mdx23c
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_mdx23c.json 2> $O/bench_mdx23c.err
python3 -c "
import json
for f in ('htdemucs','mdx23c'):
    d=json.load(open('$O/bench_'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['pcie_inclusive'], d.get('parity_rms'))
"
step done
