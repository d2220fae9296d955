#!/bin/bash
# HTDemucs fused MFMA DConv row kernel: GPU parity tests, then a same-box A/B (SESA_HTD_DCMFMA=0: the VALU row kernels)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_htdemucs.py -m gpu -x -q -rA --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gputest_dcm.txt 2>&1; rc=$?
grep -E "rms|passed|failed" gpurun_out/r06/gputest_dcm.txt | tail -8
[ $rc -eq 0 ] || exit $rc
for v in mfma valu mfma2; do
  if [ $v = valu ]; then export SESA_HTD_DCMFMA=0; else unset SESA_HTD_DCMFMA; fi
  timeout -k 10 500 python -u bench.py --model htdemucs --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/r06/dcm_bench_$v.json 2> gpurun_out/r06/dcm_bench_$v.log || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['parity_rms'], {k: v['ms_per_step'] for k, v in d['kernel_classes'].items()})" gpurun_out/r06/dcm_bench_$v.json
done
