#!/bin/bash
# Round-3 final evidence run on one MI355X, all on the tree as committed (GIT_SHA from the caller):
#   GPU parity suite, smoke, one bench line per BASELINE config (+ the bf16 throughput line and the
#   HTDemucs demucs-mode line), rocprofv3 kernel stats of the headline / configs[2] / configs[3], and the
#   sha-stamped HBM-traffic PMC summaries (separate FETCH_SIZE / WRITE_SIZE passes) that bench.py's
#   roofline.traffic reads.  Every GPU step has its own time limit; the script stops at the first failure.
set -e
O=gpurun_out/final
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[final] $(date +%T) $*"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputest.log 2>&1
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step pmc mdx23c
timeout -k 10 700 bash tools/pmc_refresh.sh mdx23c "conv3x3=conv3x3_db_kernel|tap_gemm_kernel<3, 3" \
  "tdf=tdf_dma_kernel|tdf_kernel|tdf_u_split" "act=act_split_kernel" > $O/pmc_mdx23c.log 2>&1
step pmc htdemucs
timeout -k 10 700 bash tools/pmc_refresh.sh htdemucs \
  "hconv=tok_gemm_kernel<true, 256, 128, 2, 2, 2, false, true, false>|htd_dc_conv_valu" "attn=attn_kernel" \
  > $O/pmc_htdemucs.log 2>&1
step pmc bs_roformer
timeout -k 10 700 bash tools/pmc_refresh.sh bs_roformer "tokgemm=tok_gemm" > $O/pmc_bsr.log 2>&1
step pmc scnet
timeout -k 10 700 bash tools/pmc_refresh.sh scnet "lstm=scn_lstm_mfma" > $O/pmc_scnet.log 2>&1
mkdir -p $O/pmc
cp gpurun_out/pmc_*.json $O/pmc/ 2>/dev/null || true
cp $O/pmc/pmc_*.json profiles/          # bench.py below reads the fresh, sha-matched summaries
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
step mdx23c
timeout -k 10 400 python bench.py > $O/bench_mdx23c.json 2> $O/bench_mdx23c.err
step mdx23c bf16x3
timeout -k 10 300 python bench.py --precision bf16x3 --no-cpu-baseline > $O/bench_mdx23c_bf16x3.json 2> $O/bench_mdx23c_bf16x3.err
step mdx23c fp16w2
timeout -k 10 300 python bench.py --precision fp16w2 --no-cpu-baseline > $O/bench_mdx23c_fp16w2.json 2> $O/bench_mdx23c_fp16w2.err
step mdx23c fp16 16-row tile
timeout -k 10 300 env SESA_CONV_MI4=0 python bench.py --no-cpu-baseline > $O/bench_mdx23c_fp16_mi2.json 2> $O/bench_mdx23c_fp16_mi2.err
step mdx23c fp16 again
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_mdx23c_fp16_again.json 2> $O/bench_mdx23c_fp16_again.err
step mdx23c bf16
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline > $O/bench_mdx23c_bf16.json 2> $O/bench_mdx23c_bf16.err
step bs_roformer
timeout -k 10 400 python bench.py --model bs_roformer --steps 3 --warmup 1 --cpu-sample-chunks 1 > $O/bench_bsr.json 2> $O/bench_bsr.err
step htdemucs generic
timeout -k 10 400 python bench.py --model htdemucs --steps 2 --warmup 1 --cpu-sample-chunks 2 > $O/bench_htdemucs.json 2> $O/bench_htdemucs.err
step htdemucs demucs
timeout -k 10 300 python bench.py --model htdemucs --htdemucs-mode demucs --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_htdemucs_demucsmode.json 2> $O/bench_htdemucs_demucsmode.err
step scnet
timeout -k 10 300 python bench.py --model scnet --steps 3 --warmup 1 --cpu-sample-chunks 2 > $O/bench_scnet.json 2> $O/bench_scnet.err
step ensemble
timeout -k 10 400 python bench.py --model ensemble --steps 2 --warmup 1 > $O/bench_ensemble.json 2> $O/bench_ensemble.err
step rocprof mdx23c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mdx23c -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-parity > $O/prof_mdx23c.json 2> $O/prof_mdx23c.err
step rocprof htdemucs
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_htdemucs -o run -- python3 bench.py --model htdemucs --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/prof_htdemucs.json 2> $O/prof_htdemucs.err
step rocprof bs_roformer
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bsr -o run -- python3 bench.py --model bs_roformer --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/prof_bsr.json 2> $O/prof_bsr.err
step summarize
# the raw rocpd databases are tens of MiB each: keep the per-kernel summaries, drop the raw dirs so the
# gpurun_out merge-back stays under its size cap
for r in mdx23c htdemucs bsr; do
  python3 tools/rocprof_summary.py $O/prof_$r $O/kernel_stats_$r.txt > /dev/null
  rm -rf $O/prof_$r
done
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
du -sh gpurun_out
step done
