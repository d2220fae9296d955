#!/bin/bash
# Round 5 lease Z: the one-wave iSTFT on a frame-major spectrum (the last transposed conv writes [B][T][2048][Cz];
# SESA_HTD_ISTFT_WAVE=1) -- HTDemucs GPU tests with it, same-box configs[3] bench A / B (parity) / A2, kernel trace of B.
set -e
O=gpurun_out/r05z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[r05z] $(date +%T) $*"; }
step tests wave
SESA_HTD_ISTFT_WAVE=1 timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/tests_wave.txt 2>&1 || { tail -30 $O/tests_wave.txt; exit 1; }
tail -2 $O/tests_wave.txt
step bench A fused
timeout -k 10 300 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_fused.json 2> $O/bench_fused.err
step bench B wave
SESA_HTD_ISTFT_WAVE=1 timeout -k 10 400 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_wave.json 2> $O/bench_wave.err
step bench A2 fused
timeout -k 10 300 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_fused2.json 2> $O/bench_fused2.err
step rocprof wave
SESA_HTD_ISTFT_WAVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --model htdemucs --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/prof.json 2> $O/prof.err
python3 tools/rocprof_summary.py $O/prof $O/kernel_stats_wave.txt > /dev/null
rm -rf $O/prof
grep -E "istft|ctr_kernel" $O/kernel_stats_wave.txt || true
python3 -c "
import json
for f in ('fused','wave','fused2'):
    d=json.load(open('$O/bench_'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['kernel_classes']['istft']['ms_per_step'], d['kernel_classes']['hconv']['ms_per_step'], d.get('parity_rms'))
"
step done
