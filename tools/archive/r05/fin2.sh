#!/bin/bash
# Round 5 lease FIN2: MDX23C and ensemble evidence after the execution-batch caps changed (MDX23C 2 x 85 chunks per
# forward): PMC traffic (MDX23C conv3x3 / tdf / act, the ensemble's conv3x3 -- per-launch bytes scale with the batch),
# the bench lines (configs[1] with CPU baseline and parity, repeat, bf16x3, rank-share 8; configs[4]) and the MDX23C
# kernel trace.  The HTDemucs lines follow in tools/r05/hf.sh.
set -e
O=gpurun_out/fin2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[fin2] $(date +%T) $*"; }
step pmc mdx23c
timeout -k 10 700 bash tools/pmc_refresh.sh mdx23c \
  "conv3x3=conv3x3_db_kernel<true, true, 0, false, 1, true|conv3x3_db_kernel<true, false, 0, false, 1, true" \
  "tdf=tdf_dma_kernel|tdf_kernel|tdf_u_split" "act=act_split_kernel|act_f16" > $O/pmc_mdx23c.log 2>&1
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
step pmc ensemble
timeout -k 10 900 bash tools/pmc_refresh.sh ensemble "conv3x3=conv3x3_db_kernel|tap_gemm_kernel<3, 3" > $O/pmc_ensemble.log 2>&1
rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
cp gpurun_out/pmc_*_mdx23c.json gpurun_out/pmc_conv3x3_ensemble.json profiles/
step mdx23c
timeout -k 10 400 python bench.py > $O/bench_mdx23c.json 2> $O/bench_mdx23c.err
step mdx23c again
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_mdx23c_again.json 2> $O/bench_mdx23c_again.err
step mdx23c bf16x3
timeout -k 10 300 python bench.py --precision bf16x3 --no-cpu-baseline > $O/bench_mdx23c_bf16x3.json 2> $O/bench_mdx23c_bf16x3.err
step mdx23c share8
timeout -k 10 300 python bench.py --rank-share 8 --no-cpu-baseline --no-parity > $O/bench_mdx23c_share8.json 2> $O/bench_mdx23c_share8.err
step ensemble
timeout -k 10 900 python bench.py --model ensemble --steps 2 --warmup 1 > $O/bench_ensemble.json 2> $O/bench_ensemble.err
step rocprof mdx23c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mdx23c -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/prof_mdx23c.json 2> $O/prof_mdx23c.err
python3 tools/rocprof_summary.py $O/prof_mdx23c $O/kernel_stats_mdx23c.txt > /dev/null
rm -rf $O/prof_mdx23c
python3 -c "
import json
for f in ('mdx23c','mdx23c_again','mdx23c_bf16x3','mdx23c_share8','ensemble'):
    d=json.load(open('$O/bench_'+f+'.json')); r=d['roofline']; print(f, d['value'], d['ms_per_step'], r['class'], r['frac'], r.get('traffic_over_algorithmic'), d.get('parity_rms'))
"
step done
