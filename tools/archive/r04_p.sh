#!/bin/bash
# Round 4: re-check the full-width ensemble (bench precisions) and the MDX23C parity matrix after restoring the
# conservative fp16mix plan; then the PMC passes of the final evidence run.
set -e
O=gpurun_out/final4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r04p] $(date +%T) ensemble + mdx parity"
timeout -k 10 600 python -u -m pytest tests/test_ensemble_models.py tests/test_gpu_parity.py tests/test_cli_flow.py -v -s \
  --timeout 300 --timeout-method thread -k "full_width or (levels and fp16mix) or raw_model" > $O/parity_recheck.txt 2>&1 || rc=$?
if [ "${rc:-0}" != 0 ]; then echo "[r04p] parity rc=$rc"; [ "$rc" = 1 ] || exit "$rc"; fi
PART=p bash tools/r04_final.sh
