set -o pipefail
mkdir -p gpurun_out/r06
f() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/r06/$name.txt 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/r06/$name.txt | tail -2 | cut -c1-300; return $rc; }
for v in st_pkmul st_pkadd st_pkfma st_scalar st_pkmul_nop st_pkmul_global; do
  f vs10_${v} python -u tools/victim_stress.py $v mfma 40 || exit 1
done
f vs10_pkmul_none python -u tools/victim_stress.py st_pkmul none 40
