#!/bin/bash
# Round 4: streams diagnostic 2; BS-Roformer fp16 attention with 64-query tiles for the band attention (A/B +
# parity); per-dispatch kernel trace of one BS-Roformer step.
set -e
O=gpurun_out/r04d
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04d] $(date +%T) streams diagnostic 2"
timeout -k 10 180 python tools/streams_debug2.py > $O/streams_debug2.txt 2>&1
echo "[r04d] $(date +%T) bsr parity"
timeout -k 10 600 python -u -m pytest tests/test_bsr.py tests/test_amp_precision.py -v -s --timeout 300 \
  --timeout-method thread -k "fp16 or roformer or large" > $O/parity.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04d] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
echo "[r04d] $(date +%T) bsr bench"
timeout -k 10 300 python bench.py --model bs_roformer --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_bsr.json 2> $O/bench_bsr.err
echo "[r04d] $(date +%T) bsr trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bsr -o run -- python3 bench.py --model bs_roformer --steps 1 --warmup 1 --no-cpu-baseline --no-parity > $O/prof_bsr.json 2> $O/prof_bsr.err
python3 tools/rocprof_summary.py $O/prof_bsr $O/kernel_stats_bsr.txt > /dev/null
python3 tools/trace_table.py $O/prof_bsr 0 1000000000 attn > $O/bsr_dispatches.txt 2>&1 || true
rm -rf $O/prof_bsr
echo "[r04d] $(date +%T) done"
