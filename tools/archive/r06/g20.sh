set -o pipefail
mkdir -p gpurun_out
bash tools/pmc_mfma.sh bs_roformer r06_bsr 24 && bash tools/pmc_mfma.sh mdx23c r06_mdx23c 24 && bash tools/pmc_mfma.sh htdemucs r06_htdemucs 60 && bash tools/pmc_mfma.sh scnet r06_scnet 24
for t in bsr mdx23c htdemucs scnet; do echo "== $t"; head -12 gpurun_out/pmc_r06_${t}_mfma.txt | cut -c1-200; done
