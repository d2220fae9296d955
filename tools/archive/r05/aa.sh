#!/bin/bash
# Round 5 lease AA: padded exchange buffer of the one-wave iSTFT (htd_istft_wave_kernel<PAD>) -- HTDemucs GPU tests,
# same-box configs[3] bench A (unpadded, SESA_HTD_IW_PAD=0) / B (padded, parity) / A2.
set -e
O=gpurun_out/r05aa
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { echo "[r05aa] $(date +%T) $*"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
step bench A unpadded
SESA_HTD_IW_PAD=0 timeout -k 10 300 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/bench_nopad.json 2> $O/bench_nopad.err
step bench B padded
timeout -k 10 400 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $O/bench_pad.json 2> $O/bench_pad.err
step bench A2 unpadded
SESA_HTD_IW_PAD=0 timeout -k 10 300 python bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > $O/bench_nopad2.json 2> $O/bench_nopad2.err
python3 -c "
import json
for f in ('nopad','pad','nopad2'):
    d=json.load(open('$O/bench_'+f+'.json')); k=d['kernel_classes']['istft']; print(f, d['value'], d['ms_per_step'], k['ms_per_step'], k['launches'], d.get('parity_rms'))
"
step done
