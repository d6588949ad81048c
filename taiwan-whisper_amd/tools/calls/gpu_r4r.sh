#!/bin/bash
# Round 4, call R: PMC passes over the attention forward alone (encoder self-attention shape), 16x16x32 kernel
# (ab/libtw_hip_base.so) vs the tree's 32x32x16 software-pipelined kernel: issue / wait / LDS breakdown.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4r
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for v in base cand; do
  if [ $v = base ]; then L=$R/ab/libtw_hip_base.so; else L=$R/taiwan-whisper_amd/tw/_lib/libtw_hip.so; fi
  export TW_HIP_LIB=$L
  timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $OUT/${v}_p1 -o run -- python3 $R/taiwan-whisper_amd/tools/attn_one.py > $OUT/${v}_p1.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $OUT/${v}_p2 -o run -- python3 $R/taiwan-whisper_amd/tools/attn_one.py > $OUT/${v}_p2.log 2>&1
done
ls -R $OUT | head -30
