set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for f in 512 1024 2048; do
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    tag=$(echo $grp | cut -c1-12)
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc9/f${f}_$tag -o run -- python3 $R/taiwan-whisper_amd/tools/one_gemm.py 96000 5120 1280 $f > /dev/null 2>&1
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmc9/f${f}_trace -o run -- python3 $R/taiwan-whisper_amd/tools/one_gemm.py 96000 5120 1280 $f > /dev/null 2>&1
done
echo done
