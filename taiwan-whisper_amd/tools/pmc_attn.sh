# SQ counters + kernel trace of the attention forward variants (encoder shape); run on the GPU box.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 4 8; do
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
    tag=$(echo $grp | cut -c1-12)
    TW_ATTN_FWD=$v timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmca/v${v}_$tag -o run -- python3 $R/taiwan-whisper_amd/tools/one_attn.py > /dev/null 2>&1
  done
  TW_ATTN_FWD=$v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/pmca/v${v}_trace -o run -- python3 $R/taiwan-whisper_amd/tools/one_attn.py > /dev/null 2>&1
done
echo done
