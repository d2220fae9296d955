#!/bin/bash
# Round 5 lease O: MDX23C fp16mix with the encoder level-0 TDF and the up-convs in fp16 (the new default) -- the
# four full-chunk fixtures (GPU parity tests + the bench parity leg) and a same-box A/B against the round-4 plan
# (SESA_TDF_PLAN=3333311111111111 SESA_MDX_UP16=0); the larger execution batches of BS-Roformer / SCNet / the
# ensemble with their parity legs.
set -e
O=gpurun_out/r05o
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05o] $(date +%T) tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "full_chunk_levels or parity_matrix" > $O/tests.txt 2>&1
b() {
  echo "[r05o] $(date +%T) bench $1"
  timeout -k 10 600 python bench.py $2 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
b mdx "--steps 5 --warmup 1"
SESA_TDF_PLAN=3333311111111111 SESA_MDX_UP16=0 b mdx_r4plan "--steps 5 --warmup 1 --no-parity"
b mdx2 "--steps 5 --warmup 1 --no-parity"
b bsr "--model bs_roformer --steps 3 --warmup 1"
b scn "--model scnet --steps 3 --warmup 1"
b ens "--model ensemble --steps 2 --warmup 1"
echo "[r05o] $(date +%T) done"
