# Round 5: are the SwiGLU epilogue's stores a time cost (issue / back-pressure) or a power cost (lower clock)?
# Per-dispatch effective clock and MFMA occupancy (tools/clock_pmc.py) of the production gate/up GEMM and of the
# NOSTORE probe build (scripts/gpu_r05y_swiglu_store.sh), 12 sustained calls each, one --pmc pass per build.
set -o pipefail
O=gpurun_out/${OUT:-r05z}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
cd /tmp
for v in prod NOSTORE; do
  if [ $v = prod ]; then L=""; else L=$R/build/probe/libedge_kernels_$v.so; fi
  EDGE_KERNEL_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES \
    SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $R/$O/clk_$v -o run -- \
    python3 $R/tools/kernel_probe.py --op gateup --iters 12 > $R/$O/clk_$v.log 2>&1 \
    || { echo "pmc $v failed"; tail -3 $R/$O/clk_$v.log; exit 1; }
done
cd $R
{ python tools/clock_pmc.py $O/clk_prod "gemm_4w_kernel<13" && python tools/clock_pmc.py $O/clk_NOSTORE "gemm_4w_kernel<13"; } > $O/clock.md
cat $O/clock.md
grep -h us_per_call $O/*.log
exit 0
