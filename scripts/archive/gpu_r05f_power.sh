# Round 5: is the fp32 GEMM plateau the chip's power limit?  Per-dispatch effective clock and MFMA-pipe occupancy of
# our gate/up and down GEMMs and of hipBLASLt on the same fp16 operands and K' (plain GEMM, no epilogue), each run
# back to back for 12 calls (sustained load), one --pmc pass per op.
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
cd /tmp
for op in gateup gateup_lib down down_lib; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_MFMA \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $R/$O/clk_$op -o run -- \
    python3 $R/tools/kernel_probe.py --op $op --iters 12 > $R/$O/clk_$op.log 2>&1 \
    || { echo "pmc $op failed"; tail -3 $R/$O/clk_$op.log; exit 1; }
done
cd $R
{ python tools/clock_pmc.py $O/clk_gateup "gemm_4w_kernel<13" && python tools/clock_pmc.py $O/clk_gateup_lib "Cijk" \
  && python tools/clock_pmc.py $O/clk_down "gemm_4w_kernel<10" && python tools/clock_pmc.py $O/clk_down_lib "Cijk"; } > $O/clock.md
cat $O/clock.md
grep -h us_per_call $O/*.log
exit 0
