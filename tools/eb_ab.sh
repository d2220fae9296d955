#!/bin/bash
# Round 6: execution-batch A/B at two streams, same box (bench lines without the CPU / parity legs).
set -o pipefail
O=gpurun_out/eb_ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # NAME ARGS...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-parity --no-pcie > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['config']['exec_batch'], d['config']['streams'])" $O/$n.json $n
}
run bsr_eb16 --model bs_roformer --steps 3 --warmup 1
run bsr_eb8 --model bs_roformer --steps 3 --warmup 1 --exec-batch 8
run bsr_eb16b --model bs_roformer --steps 3 --warmup 1
run mdx_eb29 --steps 3 --warmup 1
run mdx_eb43 --steps 3 --warmup 1 --exec-batch 43
run mdx_eb57 --steps 3 --warmup 1 --exec-batch 57
run mdx_eb29b --steps 3 --warmup 1
