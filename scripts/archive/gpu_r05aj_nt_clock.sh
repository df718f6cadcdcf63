# Round 5: per-dispatch clock and MFMA occupancy of the gate/up GEMM with the nontemporal SwiGLU planes (this tree;
# compare profiles/history/r05/gemm_epilogue/clock_nostore.md: plain stores 1.625 GHz / 0.671, stores off 1.738 GHz / 0.683).
set -o pipefail
O=gpurun_out/${OUT:-r05aj}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_MFMA \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $R/$O/clk_nt -o run -- \
  python3 $R/tools/kernel_probe.py --op gateup --iters 12 > $R/$O/clk_nt.log 2>&1 || { echo "pmc failed"; tail -3 $R/$O/clk_nt.log; exit 1; }
cd $R
python tools/clock_pmc.py $O/clk_nt "gemm_4w_kernel<13" > $O/clock.md
cat $O/clock.md
rm -rf $O/clk_nt
exit 0
