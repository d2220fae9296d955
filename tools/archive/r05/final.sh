#!/bin/bash
# Round-5 final evidence run on one MI355X, on the tree as committed:
#   GPU parity suite, smoke, sha-stamped HBM-traffic PMC summaries (separate FETCH_SIZE / WRITE_SIZE passes) for the
#   dominant classes + the streaming classes, one bench line per BASELINE config (+ rank-share rehearsals), rocprofv3
#   kernel stats.  Every GPU step has its own time limit; the script stops at the first crash or time limit.
#   PART=t|p|b|c splits it over calls (t: GPU tests + smoke, p: PMC passes, b: bench lines, c: rocprof).
#   Second pass (final5b) after the round's last source changes: the PMC step re-measures only the classes whose
#   sha stamps the changes invalidated (MDX23C conv3x3 / tdf / act, HTDemucs hconv / simt / attn, the ensemble's
#   conv3x3); the BS-Roformer, SCNet and streaming-class summaries still match the tree.
set -e
O=gpurun_out/final5b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[final] $(date +%T) $*"; }
PART=${PART:-tpbc}
if [[ $PART == *t* ]]; then
step tests
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 || rc=$?
# plain test failures (exit 1) are reported and the evidence run goes on; a crash / time limit stops it
if [ "${rc:-0}" != 0 ]; then echo "[final] tests rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
if [[ $PART == *p* ]]; then
step pmc mdx23c
timeout -k 10 700 bash tools/pmc_refresh.sh mdx23c \
  "conv3x3=conv3x3_db_kernel<true, true, 0, false, 1, true|conv3x3_db_kernel<true, false, 0, false, 1, true" \
  "tdf=tdf_dma_kernel|tdf_kernel|tdf_u_split" "act=act_split_kernel|act_f16" > $O/pmc_mdx23c.log 2>&1
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
step pmc htdemucs
timeout -k 10 700 bash tools/pmc_refresh.sh htdemucs \
  "hconv=2, false, true, false|1, false, true, false|htd_rw3|htd_ctr" \
  "simt=htd_dc_|htd_item_stats|htd_gn_apply|htd_norm_freq|htd_norm_time" \
  "attn=attn_kernel|attn_f16_kernel" > $O/pmc_htdemucs.log 2>&1
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
step pmc ensemble
timeout -k 10 900 bash tools/pmc_refresh.sh ensemble "conv3x3=conv3x3_db_kernel|tap_gemm_kernel<3, 3" > $O/pmc_ensemble.log 2>&1
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
mkdir -p $O/pmc
cp gpurun_out/pmc_*.json $O/pmc/ 2>/dev/null || true
cp $O/pmc/pmc_*.json profiles/          # bench.py below reads the fresh, sha-matched summaries
fi
if [[ $PART == *b* ]]; then
[ -d $O/pmc ] && cp $O/pmc/pmc_*.json profiles/ 2>/dev/null || true
step mdx23c
timeout -k 10 400 python bench.py > $O/bench_mdx23c.json 2> $O/bench_mdx23c.err
step mdx23c again
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_mdx23c_again.json 2> $O/bench_mdx23c_again.err
step mdx23c bf16x3
timeout -k 10 300 python bench.py --precision bf16x3 --no-cpu-baseline > $O/bench_mdx23c_bf16x3.json 2> $O/bench_mdx23c_bf16x3.err
step mdx23c share8
timeout -k 10 300 python bench.py --rank-share 8 --no-cpu-baseline --no-parity > $O/bench_mdx23c_share8.json 2> $O/bench_mdx23c_share8.err
step bs_roformer
timeout -k 10 600 python bench.py --model bs_roformer --steps 3 --warmup 1 --cpu-sample-chunks 8 > $O/bench_bsr.json 2> $O/bench_bsr.err
step htdemucs
timeout -k 10 600 python bench.py --model htdemucs --steps 2 --warmup 1 --cpu-sample-chunks 8 > $O/bench_htdemucs.json 2> $O/bench_htdemucs.err
step htdemucs share8
timeout -k 10 300 python bench.py --model htdemucs --rank-share 8 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_htdemucs_share8.json 2> $O/bench_htdemucs_share8.err
step scnet
timeout -k 10 600 python bench.py --model scnet --steps 3 --warmup 1 --cpu-sample-chunks 8 > $O/bench_scnet.json 2> $O/bench_scnet.err
step ensemble
timeout -k 10 900 python bench.py --model ensemble --steps 2 --warmup 1 > $O/bench_ensemble.json 2> $O/bench_ensemble.err
fi
if [[ $PART == *c* ]]; then
step rocprof mdx23c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mdx23c -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/prof_mdx23c.json 2> $O/prof_mdx23c.err
step rocprof htdemucs
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_htdemucs -o run -- python3 bench.py --model htdemucs --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/prof_htdemucs.json 2> $O/prof_htdemucs.err
step rocprof bs_roformer
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bsr -o run -- python3 bench.py --model bs_roformer --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/prof_bsr.json 2> $O/prof_bsr.err
step rocprof scnet
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_scnet -o run -- python3 bench.py --model scnet --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/prof_scnet.json 2> $O/prof_scnet.err
step summarize
for r in mdx23c htdemucs bsr scnet; do
  python3 tools/rocprof_summary.py $O/prof_$r $O/kernel_stats_$r.txt > /dev/null
  rm -rf $O/prof_$r
done
fi
du -sh gpurun_out
step done
