#!/bin/bash
# Round 4: HTDemucs fp16 conv gathers with PD register sets (SESA_HCONV_PD = 1 / 2 / 3): parity, same-box A/B;
# per-kernel stats of one fp16mix HTDemucs step; BS-Roformer with the half tile as default.
set -e
O=gpurun_out/r04i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04i] $(date +%T) parity (PD 2 / 3)"
for pd in 2 3; do
  SESA_HCONV_PD=$pd timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -v -s --timeout 300 \
    --timeout-method thread -k "full_segment or small_matches" > $O/parity_pd$pd.txt 2>&1 || rc=$?
  if [ "${rc:-0}" != 0 ]; then echo "[r04i] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
done
run() {
  echo "[r04i] $(date +%T) $1"
  timeout -k 10 300 env $2 python bench.py $3 --no-cpu-baseline > $O/bench_$1.json 2> $O/bench_$1.err
}
run htd_pd1 SESA_HCONV_PD=1 "--model htdemucs --steps 1 --warmup 1"
run htd_pd2 SESA_HCONV_PD=2 "--model htdemucs --steps 1 --warmup 1"
run htd_pd3 SESA_HCONV_PD=3 "--model htdemucs --steps 1 --warmup 1"
run htd_pd1b SESA_HCONV_PD=1 "--model htdemucs --steps 1 --warmup 1"
run bsr fp=1 "--model bs_roformer --steps 2 --warmup 1"
echo "[r04i] $(date +%T) htdemucs trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_htd -o run -- python3 bench.py --model htdemucs --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $O/prof_htd.json 2> $O/prof_htd.err
python3 tools/rocprof_summary.py $O/prof_htd $O/kernel_stats_htd.txt > /dev/null
rm -rf $O/prof_htd
echo "[r04i] $(date +%T) done"
