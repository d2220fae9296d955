set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --model bs_roformer --steps 1 --warmup 0 --track-seconds 24 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/pmc_bsr_sq -o run -- $B > gpurun_out/pmc_bsr_sq.json 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_bsr_f -o run -- $B > /dev/null 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_bsr_w -o run -- $B > /dev/null 2>&1
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_bsr_h -o run -- $B > /dev/null 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bsr -o run -- $B > gpurun_out/prof_bsr.json 2>&1
python3 tools/pmc_sq.py gpurun_out/pmc_bsr_sq gpurun_out/pmc_bsr_h > gpurun_out/pmc_bsr_sq.txt
python3 tools/pmc_traffic.py gpurun_out/pmc_bsr_f gpurun_out/pmc_bsr_w "tok_gemm_kernel" gpurun_out/pmc_tokgemm.json
python3 tools/rocprof_summary.py gpurun_out/prof_bsr gpurun_out/prof_bsr_summary.txt
