#!/bin/bash
# Re-stamp the token-GEMM-class PMC summaries (tokgemm / attn / hconv / lstm) after a sesa_tokgemm change,
# and re-run the BS-Roformer / HTDemucs / SCNet / ensemble bench lines on the same tree.
set -e
O=gpurun_out/refresh
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[refresh] $(date +%T) $*"; }
step parity values
timeout -k 10 300 python -u -m pytest tests/test_bsr.py tests/test_ensemble_models.py -m gpu -x -s -q --timeout 150 \
  --timeout-method thread -k "fp16 or ensemble" > $O/parity_fp16_s.log 2>&1
step pmc htdemucs
timeout -k 10 700 bash tools/pmc_refresh.sh htdemucs \
  "hconv=tok_gemm_kernel<true, 256, 128, 2, 2, 2, false, true, false>|htd_dc_conv_valu" "attn=attn_kernel" \
  > $O/pmc_htdemucs.log 2>&1
step pmc bs_roformer
timeout -k 10 700 bash tools/pmc_refresh.sh bs_roformer "tokgemm=tok_gemm" > $O/pmc_bsr.log 2>&1
step pmc scnet
timeout -k 10 700 bash tools/pmc_refresh.sh scnet "lstm=scn_lstm_mfma" > $O/pmc_scnet.log 2>&1
mkdir -p $O/pmc
cp gpurun_out/pmc_hconv.json gpurun_out/pmc_tokgemm.json gpurun_out/pmc_attn.json gpurun_out/pmc_lstm.json $O/pmc/
cp $O/pmc/pmc_*.json profiles/
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
step bs_roformer
timeout -k 10 400 python bench.py --model bs_roformer --steps 3 --warmup 1 --cpu-sample-chunks 1 > $O/bench_bsr.json 2> $O/bench_bsr.err
step htdemucs
timeout -k 10 400 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_htdemucs.json 2> $O/bench_htdemucs.err
step scnet
timeout -k 10 300 python bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_scnet.json 2> $O/bench_scnet.err
step ensemble
timeout -k 10 400 python bench.py --model ensemble --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_ensemble.json 2> $O/bench_ensemble.err
step mdx23c
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_mdx23c.json 2> $O/bench_mdx23c.err
step done
