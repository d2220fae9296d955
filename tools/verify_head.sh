set -e
O=gpurun_out/v1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[v] $(date +%T) tests"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gputest.log 2>&1
echo "[v] $(date +%T) smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "[v] $(date +%T) mdx"
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_mdx23c.json 2> $O/bench_mdx23c.err
echo "[v] $(date +%T) bsr"
timeout -k 10 400 python bench.py --model bs_roformer --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_bsr.json 2> $O/bench_bsr.err
echo "[v] $(date +%T) done"
