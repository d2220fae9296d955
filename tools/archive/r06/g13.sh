set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06/gputest_g13.txt 2>&1; rc=$?
tail -5 gpurun_out/r06/gputest_g13.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke_g13.txt 2>&1; rc=$?
tail -3 gpurun_out/r06/smoke_g13.txt; exit $rc
