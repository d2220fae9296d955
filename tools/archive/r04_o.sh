#!/bin/bash
# Round 4: confirm HTDemucs after reverting the DConv-apply batching (iSTFT XCD grid + float4 embedding add kept);
# smoke in fp16mix.
set -e
O=gpurun_out/r04o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04o] $(date +%T) smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "[r04o] $(date +%T) htd"
timeout -k 10 300 python bench.py --model htdemucs --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_htd.json 2> $O/bench_htd.err
echo "[r04o] $(date +%T) done"
