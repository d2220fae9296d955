#!/bin/bash
set -e
O=gpurun_out/be
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python bench.py --model bs_roformer --steps 3 --warmup 1 --cpu-sample-chunks 1 > $O/bench_bsr.json 2> $O/bench_bsr.err
timeout -k 10 400 python bench.py --model ensemble --steps 2 --warmup 1 > $O/bench_ensemble.json 2> $O/bench_ensemble.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_bsr -o run -- python3 bench.py --model bs_roformer --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/prof_bsr.json 2> $O/prof_bsr.err
python3 tools/rocprof_summary.py $O/prof_bsr $O/kernel_stats_bsr.txt > /dev/null
rm -rf $O/prof_bsr
