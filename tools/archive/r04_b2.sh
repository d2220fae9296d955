#!/bin/bash
# Round-4 final evidence, secondary bench lines (the MDX23C lines ran in PART=b of r04_final.sh): BS-Roformer,
# HTDemucs, SCNet, ensemble, each with an 8-chunk CPU leg (progress on stderr).
set -e
O=gpurun_out/final4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[final] $(date +%T) $*"; }
[ -d $O/pmc ] && cp $O/pmc/pmc_*.json profiles/ 2>/dev/null || true
step bs_roformer
timeout -k 10 600 python bench.py --model bs_roformer --steps 3 --warmup 1 --cpu-sample-chunks 8 > $O/bench_bsr.json 2> $O/bench_bsr.err
step htdemucs generic
timeout -k 10 600 python bench.py --model htdemucs --steps 2 --warmup 1 --cpu-sample-chunks 8 > $O/bench_htdemucs.json 2> $O/bench_htdemucs.err
step scnet
timeout -k 10 600 python bench.py --model scnet --steps 3 --warmup 1 --cpu-sample-chunks 8 > $O/bench_scnet.json 2> $O/bench_scnet.err
step ensemble
timeout -k 10 600 python bench.py --model ensemble --steps 2 --warmup 1 > $O/bench_ensemble.json 2> $O/bench_ensemble.err
step done
