#!/bin/bash
# Round 5 lease N: execution-batch sweep (chunks per forward) for HTDemucs / MDX23C / BS-Roformer against the planner
# defaults (EXEC_CAP); HTDemucs transposed convs on htd_ctr_kernel vs the token GEMM (SESA_HTD_CTR=0) and the
# vectorised GroupNorm apply vs the scalar one (SESA_HTD_STATS4=0); HTDemucs GPU tests first.
set -e
O=gpurun_out/r05n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05n] $(date +%T) tests"
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.txt 2>&1
b() {
  echo "[r05n] $(date +%T) bench $1"
  timeout -k 10 400 python bench.py $2 --no-cpu-baseline --no-parity > $O/bench_$1.json 2> $O/bench_$1.err
}
b htd "--model htdemucs --steps 3 --warmup 1"
SESA_HTD_CTR=0 b htd_noctr "--model htdemucs --steps 3 --warmup 1"
b htd_eb64 "--model htdemucs --steps 3 --warmup 1 --exec-batch 64"
b htd_eb48 "--model htdemucs --steps 3 --warmup 1 --exec-batch 48"
SESA_HTD_STATS4=0 b htd_oldnorm "--model htdemucs --steps 3 --warmup 1"
b mdx "--steps 5 --warmup 1"
b mdx_eb85 "--steps 5 --warmup 1 --exec-batch 85"
b bsr "--model bs_roformer --steps 3 --warmup 1"
b bsr_eb8 "--model bs_roformer --steps 3 --warmup 1 --exec-batch 8"
b bsr_eb16 "--model bs_roformer --steps 3 --warmup 1 --exec-batch 16"
b scn "--model scnet --steps 3 --warmup 1"
b scn_eb96 "--model scnet --steps 3 --warmup 1 --exec-batch 96"
echo "[r05n] $(date +%T) done"
