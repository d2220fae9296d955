#!/bin/bash
# Round 5 lease V: the one-wave-per-signal iSTFT (htd_istft_wave_kernel, SESA_HTD_ISTFT_WAVE=1) -- HTDemucs GPU tests
# with it, then same-box configs[3] bench A (fused) / B (wave, with the parity fixtures) / A2, and a kernel-trace of B.
set -e
O=gpurun_out/r05v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[r05v] $(date +%T) $*"; }
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
SESA_HTD_ISTFT_WAVE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --model htdemucs --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/prof.json 2> $O/prof.err
python3 tools/rocprof_summary.py $O/prof $O/kernel_stats_wave.txt > /dev/null
rm -rf $O/prof
head -8 $O/kernel_stats_wave.txt
grep istft $O/kernel_stats_wave.txt || true
step done
