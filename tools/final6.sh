#!/bin/bash
# Round-6 final evidence run on one MI355X, on the tree as committed:
#   t: the GPU parity suite + smoke;
#   p: sha-stamped HBM-traffic PMC summaries (separate FETCH_SIZE / WRITE_SIZE passes, tools/pmc_refresh.sh) for
#      every class a bench line may name as dominant, copied into profiles/ for bench.py;
#   b: one bench line per BASELINE config (+ the owned-form rank-share rehearsals);
#   c: rocprofv3 kernel-trace stats per model.
# Every GPU step has its own time limit; the script stops at the first crash or time limit.
#   PART=t|p|b|c (any combination) selects the parts, one gpurun call each.
set -e
O=gpurun_out/final6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[final6] $(date +%T) $*"; }
PART=${PART:-tpbc}
if [[ $PART == *t* ]]; then
  step tests
  rc=0
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $O/gputest.log 2>&1 || rc=$?
  tail -3 $O/gputest.log
  # plain test failures (exit 1) are reported and the evidence run goes on; a crash / time limit stops it
  if [ "$rc" != 0 ]; then echo "[final6] tests rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -2 $O/smoke.log
fi
if [[ $PART == *p* ]]; then
  pmc() {  # MODEL SPEC...   (PMC_MODELS="a b ..." runs only those)
    local m=$1; shift
    [ -z "$PMC_MODELS" ] || [[ " $PMC_MODELS " == *" $m "* ]] || return 0
    step pmc $m
    timeout -k 10 800 bash tools/pmc_refresh.sh $m "$@" > $O/pmc_$m.log 2>&1
    if [ $m = mdx23c ]; then   # the streaming classes (STFT / iSTFT / gather + OLA) from the same two passes
      timeout -k 10 120 python3 tools/pmc_stream.py gpurun_out/pmc_mdx23c_f gpurun_out/pmc_mdx23c_w mdx23c \
        "$(python3 -c 'import bench; print(bench.default_precision("mdx23c"))')" gpurun_out > $O/pmc_stream.log 2>&1
    fi
    rm -rf gpurun_out/pmc_*_f gpurun_out/pmc_*_w
  }
  pmc mdx23c "conv3x3=conv3x3_db_kernel<true, true, 0, false, 1, true|conv3x3_db_kernel<true, false, 0, false, 1, true" \
    "tdf=tdf_dma_kernel|tdf_kernel|tdf_u_split" "act=act_split_kernel|act_f16"
  pmc bs_roformer "tokgemm=tok_gemm_glds_kernel|tok_gemm_kernel" "attn=attn_f16_kernel|attn_f16_band_kernel|attn_kernel"
  pmc scnet "lstm=scn_lstm" "tokgemm=tok_gemm_glds_kernel|tok_gemm_kernel" "simt=scn_cm_|scn_gelu_rows"
  pmc htdemucs "hconv=2, false, true, false|1, false, true, false|htd_rw3|htd_ctr" \
    "simt=htd_dc_|htd_item_stats|htd_gn_apply|htd_norm_freq|htd_norm_time" "attn=attn_kernel|attn_f16_kernel"
  pmc ensemble "conv3x3=conv3x3_db_kernel|tap_gemm_kernel<3, 3" "tokgemm=tok_gemm_glds_kernel|tok_gemm_kernel"
  mkdir -p $O/pmc
  cp gpurun_out/pmc_*_*.json gpurun_out/pmc_stft.json gpurun_out/pmc_istft.json gpurun_out/pmc_ola.json $O/pmc/ \
    2>/dev/null || true
  ls $O/pmc
fi
if [[ $PART == *b* ]]; then
  [ -d $O/pmc ] && cp $O/pmc/pmc_*.json profiles/ 2>/dev/null || true
  line() {  # NAME SECONDS ARGS...   (LINES="a b ..." runs only those)
    local n=$1 s=$2; shift 2
    [ -z "$LINES" ] || [[ " $LINES " == *" $n "* ]] || return 0
    step bench $n
    timeout -k 10 $s python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err
    python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d['roofline']
print(sys.argv[2], d['value'], d['ms_per_step'], r['class'], r['frac'], r.get('traffic_over_algorithmic'), d.get('parity_rms'),
      (d.get('pcie_inclusive') or {}).get('value'), (d.get('cpu_baseline') or {}).get('value'))" $O/bench_$n.json $n
  }
  line mdx23c 500
  line mdx23c_share8 300 --rank-share 8 --no-cpu-baseline --no-parity
  line bs_roformer 600 --model bs_roformer --steps 3 --warmup 1 --cpu-sample-chunks 8
  line scnet 600 --model scnet --steps 3 --warmup 1 --cpu-sample-chunks 8
  line htdemucs 700 --model htdemucs --steps 2 --warmup 1 --cpu-sample-chunks 8
  line htdemucs_share8 300 --model htdemucs --rank-share 8 --steps 3 --warmup 1 --no-cpu-baseline --no-parity
  line ensemble 900 --model ensemble --steps 2 --warmup 1
  line ensemble_streams2 600 --model ensemble --steps 2 --warmup 1 --streams 2 --no-cpu-baseline --no-parity
fi
if [[ $PART == *c* ]]; then
  prof() {  # NAME ARGS...
    local n=$1; shift
    step rocprof $n
    # --streams 1: the kernel averages then match the single-stream pass the bench line's roofline is timed on
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run -- python3 bench.py "$@" --streams 1 --no-cpu-baseline \
      --no-parity --no-pcie > $O/prof_$n.json 2> $O/prof_$n.err
    python3 tools/rocprof_summary.py $O/prof_$n $O/kernel_stats_$n.txt > /dev/null
    rm -rf $O/prof_$n
  }
  prof mdx23c --steps 4 --warmup 1
  prof bsr --model bs_roformer --steps 1 --warmup 1
  prof scnet --model scnet --steps 1 --warmup 1
  prof htdemucs --model htdemucs --steps 1 --warmup 1
fi
du -sh gpurun_out
step done
