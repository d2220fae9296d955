set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_scnet.py tests/test_ensemble_models.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gputest_g16.txt 2>&1; rc=$?
tail -4 gpurun_out/r06/gputest_g16.txt
[ $rc -eq 0 ] || exit $rc
for v in mfma valu; do
  if [ $v = valu ]; then export SESA_SCN_CM_VALU=1; else unset SESA_SCN_CM_VALU; fi
  timeout -k 10 400 python -u bench.py --model scnet --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > gpurun_out/r06/g16_bench_scnet_$v.json 2> gpurun_out/r06/g16_bench_scnet_$v.log || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/r06/g16_bench_scnet_$v.json
done
unset SESA_SCN_CM_VALU
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_g16 -o scn -- python3 -u bench.py --model scnet --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-pcie > gpurun_out/r06/g16_prof.log 2>&1
