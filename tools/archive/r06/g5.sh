set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; tail -1 gpurun_out/r06/$name.txt | cut -c1-300; return $rc; }
for k in 99 0 1 2 3 4 5 6 7; do
  f fs5_only$k env SESA_DEBUG_ONLY=$k python -u tools/fft_stress.py mdx23c bf16x3 200 || exit 1
done
