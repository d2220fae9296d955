set -o pipefail
mkdir -p gpurun_out/r06
for m in htdemucs mdx23c; do
  for rs in 0 8; do
    timeout -k 10 500 python -u bench.py --model $m --steps 3 --warmup 1 --no-cpu-baseline --no-parity --rank-share $rs > gpurun_out/r06/g15_${m}_rs$rs.json 2> gpurun_out/r06/g15_${m}_rs$rs.log || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['pcie_inclusive'])" gpurun_out/r06/g15_${m}_rs$rs.json
  done
done
