# PMC passes (kernel counters only, no trace domains) over the fp32-mode bench kernels: attention, QKV, colsum, norm.
# env: OPS (default "attn qkv colsum norm"), OUT (dir under gpurun_out)
set -o pipefail
OUT=${OUT:-pmc_fp32}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for op in ${OPS:-attn qkv colsum norm}; do
  timeout -k 10 120 python tools/kernel_probe.py --op $op > gpurun_out/$OUT/time_$op.log 2>&1 || { echo "time $op failed"; tail gpurun_out/$OUT/time_$op.log; exit 1; }
  tail -1 gpurun_out/$OUT/time_$op.log
done
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for op in ${OPS:-attn qkv colsum norm}; do
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/p${i}_$op -o run -- python $GRAFT_REPO_ROOT/tools/kernel_probe.py --op $op --iters 5 > $GRAFT_REPO_ROOT/gpurun_out/$OUT/p${i}_$op.log 2>&1 || { echo "pmc $i $op failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/$OUT/p${i}_$op.log; exit 1; }
  done
done
echo pmc done
