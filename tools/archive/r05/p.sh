#!/bin/bash
# Round 5 lease P: the configs[4] line's dominant class is now conv3x3 (the MDX23C member in bf16x3): its PMC traffic
# summary on the ensemble workload, then the ensemble bench line again (no CPU baseline) to carry it.
set -e
O=gpurun_out/r05p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05p] $(date +%T) pmc ensemble"
timeout -k 10 900 bash tools/pmc_refresh.sh ensemble "conv3x3=conv3x3_db_kernel|tap_gemm_kernel<3, 3" > $O/pmc_ensemble.log 2>&1
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
cp gpurun_out/pmc_conv3x3_ensemble.json profiles/
echo "[r05p] $(date +%T) bench ensemble"
timeout -k 10 900 python bench.py --model ensemble --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_ensemble.json 2> $O/bench_ensemble.err
echo "[r05p] $(date +%T) done"
