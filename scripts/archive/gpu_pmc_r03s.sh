# PMC passes (kernel counters only, no trace domains) over the fp32 bench kernels at the bench shape, current build:
# the plane-staged attention (KVP), the QKV GEMM with K / V^T planes, RMSNorm.  Summary: tools/pmc_ops.py.
set -o pipefail
OUT=pmc_r03s
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for op in attn qkv norm; do
  timeout -k 10 120 python tools/kernel_probe.py --op $op --kv-planes 1 > gpurun_out/$OUT/time_$op.log 2>&1 || { echo "time $op failed"; tail gpurun_out/$OUT/time_$op.log; exit 1; }
  tail -1 gpurun_out/$OUT/time_$op.log
done
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for op in attn qkv norm; do
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/$OUT/p${i}_$op -o run -- python $R/tools/kernel_probe.py --op $op --kv-planes 1 --iters 5 > $R/gpurun_out/$OUT/p${i}_$op.log 2>&1 || { echo "pmc $i $op failed"; tail -3 $R/gpurun_out/$OUT/p${i}_$op.log; exit 1; }
  done
done
cd $R
python tools/pmc_ops.py gpurun_out/$OUT > gpurun_out/$OUT/summary.md && cat gpurun_out/$OUT/summary.md
exit 0
