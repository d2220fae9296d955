#!/bin/bash
# Round 5 lease AB: the whole GPU parity suite + smoke on the final tree (after the HTDemucs frame-major iSTFT default).
set -e
O=gpurun_out/r05ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[r05ab] $(date +%T) tests"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
echo "[r05ab] $(date +%T) smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
echo "[r05ab] $(date +%T) done"
