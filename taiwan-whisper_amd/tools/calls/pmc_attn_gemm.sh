#!/bin/bash
# Limiter study of the attention forward (tools/attn_one.py, encoder shape) and of the persistent GEMM (tools/one_gemm.py,
# encoder fc1 shape): three --pmc passes each (<= 8 SQ counters + GRBM_GUI_ACTIVE), one kernel trace each.
# Summaries: python tools/pmc_kernel.py <regex> gpurun_out/pmc5/<tag>_p*
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc5
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
P3="SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F SQ_INSTS_VALU_ADD_F SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
run() {  # tag, then the program
  tag=$1; shift
  timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${tag}_trace -o run -- "$@" > $OUT/${tag}_trace.log 2>&1 || return 1
  i=1
  for P in "$P1" "$P2" "$P3"; do
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/${tag}_p$i -o run -- "$@" > $OUT/${tag}_p$i.log 2>&1 || return 1
    i=$((i+1))
  done
}
run attn python3 $R/taiwan-whisper_amd/tools/attn_one.py --reps 5 || exit 1
echo "attn passes done"
run gemm python3 $R/taiwan-whisper_amd/tools/one_gemm.py 96000 5120 1280 || exit 1
echo "gemm passes done"
cd $R
python3 taiwan-whisper_amd/tools/pmc_kernel.py attn_fwd $OUT/attn_p1 $OUT/attn_p2 $OUT/attn_p3 > $OUT/attn_summary.txt
python3 taiwan-whisper_amd/tools/pmc_kernel.py gemm_pp $OUT/gemm_p1 $OUT/gemm_p2 $OUT/gemm_p3 > $OUT/gemm_summary.txt
cat $OUT/attn_summary.txt $OUT/gemm_summary.txt
