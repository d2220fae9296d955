#!/bin/bash
# Round-4 final evidence after the last token-GEMM / attention change: PMC passes for the classes compiled from
# sesa_tokgemm.hip (BS-Roformer tokgemm / attn, HTDemucs hconv / attn), then the BS-Roformer, HTDemucs and
# ensemble bench lines and their kernel stats.
set -e
O=gpurun_out/final4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[final] $(date +%T) $*"; }
step pmc htdemucs
timeout -k 10 700 bash tools/pmc_refresh.sh htdemucs "hconv=2, false, true, false|1, false, true, false|htd_dc_conv_valu" \
  "attn=attn_kernel|attn_f16_kernel" > $O/pmc_htdemucs2.log 2>&1
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
step pmc bs_roformer
timeout -k 10 700 bash tools/pmc_refresh.sh bs_roformer "tokgemm=tok_gemm" > $O/pmc_bsr2.log 2>&1
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
mkdir -p $O/pmc2
cp gpurun_out/pmc_tokgemm.json gpurun_out/pmc_hconv.json $O/pmc2/
cp $O/pmc2/pmc_*.json profiles/
step bs_roformer
timeout -k 10 600 python bench.py --model bs_roformer --steps 3 --warmup 1 --cpu-sample-chunks 8 > $O/bench_bsr2.json 2> $O/bench_bsr2.err
step htdemucs
timeout -k 10 600 python bench.py --model htdemucs --steps 2 --warmup 1 --cpu-sample-chunks 8 > $O/bench_htdemucs2.json 2> $O/bench_htdemucs2.err
step ensemble
timeout -k 10 600 python bench.py --model ensemble --steps 2 --warmup 1 > $O/bench_ensemble2.json 2> $O/bench_ensemble2.err
step done
