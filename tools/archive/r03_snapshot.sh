#!/bin/bash
# Round-3 evidence run on one MI355X: GPU parity suite, smoke, one bench line per BASELINE config
# (+ the bf16 throughput line and the HTDemucs demucs-mode line), rocprofv3 kernel stats of the
# headline.  Every GPU step has its own time limit; the script stops at the first failure.
set -e
O=gpurun_out/snap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[snapshot] $(date +%T) $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputest.log 2>&1
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step mdx23c
timeout -k 10 400 python bench.py > $O/bench_mdx23c.json 2> $O/bench_mdx23c.err
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
step done
