#!/bin/bash
# A/B of the persistent forward GEMM kernels on the encoder fc1 shape (96000 x 5120 x 1280): the 4-slot ring
# (flags 2048) against the two-buffer ping-pong (flags 2048 | 1 << 21): timing + identity (tools/bench_ring.py),
# then per variant a kernel trace and two --pmc passes (SQ stalls / VMEM issue; TA / TCP / TD pipe).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc5r
mkdir -p $OUT
timeout -k 10 300 python3 -u $R/taiwan-whisper_amd/tools/bench_ring.py 3 > $OUT/bench_ring.log 2>&1 || { cat $OUT/bench_ring.log; exit 1; }
cat $OUT/bench_ring.log
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_TCR_TCP_STALL_CYCLES TCP_PENDING_STALL_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE"
for v in ring:2048 pp2:2099200; do
  tag=${v%%:*}; fl=${v#*:}
  timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $OUT/${tag}_p1 -o run -- python3 $R/taiwan-whisper_amd/tools/one_gemm.py 96000 5120 1280 $fl > $OUT/${tag}_p1.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $OUT/${tag}_p2 -o run -- python3 $R/taiwan-whisper_amd/tools/one_gemm.py 96000 5120 1280 $fl > $OUT/${tag}_p2.log 2>&1 || exit 1
done
cd $R
for tag in ring pp2; do
  k=gemm_ring; [ $tag = pp2 ] && k=gemm_pp
  echo "== $tag"; python3 taiwan-whisper_amd/tools/pmc_kernel.py $k $OUT/${tag}_p1 $OUT/${tag}_p2 | tee $OUT/${tag}_summary.txt
done
