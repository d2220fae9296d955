set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/r06/$name.txt | tail -4 | cut -c1-300; return $rc; }
for a in mfma atomic64 atomic32 lds epilogue; do
  f fs7_$a python -u tools/fft_stress.py agg:$a x 200 || exit 1
done
