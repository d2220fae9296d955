#!/bin/bash
# BS-Roformer full vocals config: which launch first differs when forwards run on two streams (per-launch checksums)
set -o pipefail
mkdir -p gpurun_out/r06
STREAMS_TRACE_CONFIG=config_bs_roformer_vocals.yaml timeout -k 10 600 python -u tools/streams_trace.py bs_roformer fp16 2 6 0 10584000 > gpurun_out/r06/st_bsr_full.txt 2>&1; rc=$?
grep -v "^W2026" gpurun_out/r06/st_bsr_full.txt | tail -25 | cut -c1-400; exit $rc
