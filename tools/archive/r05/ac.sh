#!/bin/bash
# Round 5 lease AC: window in LDS + time-branch prefetch in the one-wave iSTFT (htd_istft_wave_kernel<PF>) -- HTDemucs GPU tests,
# same-box configs[3] bench A (nopf, SESA_HTD_IW_PF=0) / B (pf, parity) / A2.
set -e
O=gpurun_out/r05ac
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[r05ac] $(date +%T) $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
step bench A nopf
SESA_HTD_IW_PF=0 timeout -k 10 300 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/bench_nopf.json 2> $O/bench_nopf.err
step bench B pf
timeout -k 10 400 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $O/bench_pf.json 2> $O/bench_pf.err
step bench A2 nopf
SESA_HTD_IW_PF=0 timeout -k 10 300 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/bench_nopf2.json 2> $O/bench_nopf2.err
python3 -c "
import json
for f in ('nopf','pf','nopf2'):
    d=json.load(open('$O/bench_'+f+'.json')); k=d['kernel_classes']['istft']; print(f, d['value'], d['ms_per_step'], k['ms_per_step'], k['launches'], d.get('parity_rms'))
"
step done
