# Round 6: effective clock and MFMA-pipe occupancy of the fp32 bench step's kernels (final tree): one rocprofv3 --pmc pass
# (kernel counters only) over a short bench, summarised per kernel by tools/clock_pmc.py.
set -o pipefail
O=gpurun_out/${OUT:-r06k}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/pmc -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-bf16 --no-fp32-weights --no-hf-compare --no-sweep > $R/$O/pmc.log 2>&1) || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
for k in "gemm_4w_kernel<13" "gemm_4w_kernel<10" "gemm_4w_kernel<14" "flash_attn_fwd_x6" "rmsnorm_f32" "gemm_4w_kernel<15"; do
  python tools/clock_pmc.py $O/pmc "$k" | grep -E "dispatches|median"
done > $O/clock_summary.md
cat $O/clock_summary.md
exit 0
