#!/bin/bash
# Round 4: HTDemucs iSTFT frames on an XCD-grouped grid, vectorised frequency-embedding add, DConv apply with
# batched residual loads: parity + bench (+ per-kernel stats); MDX23C bench (up16 default) once more.
set -e
O=gpurun_out/r04n
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04n] $(date +%T) parity"
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -v -s --timeout 300 --timeout-method thread \
  -k "full_segment or small_matches or demucs_mode or batch" > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04n] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
run() {
  echo "[r04n] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run htd fp=1 "--model htdemucs --steps 1 --warmup 1"
run htd_b fp=1 "--model htdemucs --steps 1 --warmup 1"
echo "[r04n] $(date +%T) trace"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_htd -o run -- python3 bench.py --model htdemucs --steps 1 --warmup 0 --track-seconds 600 --no-cpu-baseline --no-parity > $O/prof_htd.log 2>&1
python3 tools/rocprof_summary.py $O/prof_htd $O/kernel_stats_htd600.txt > /dev/null || true
rm -rf $O/prof_htd
echo "[r04n] $(date +%T) done"
