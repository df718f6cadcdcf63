# Round 6: PMC passes (kernel counters only) of the fp32 QKV GEMM (bench path: K / V^T planes) against the gate/up GEMM:
# where the QKV's waves wait (it is the least MFMA-busy GEMM of the step).
set -o pipefail
O=${OUT:-r06n}
mkdir -p gpurun_out/$O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for op in qkv gateup; do
    kv=""; [ $op = qkv ] && kv="--kv-planes 1"
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/$O/p${i}_$op -o run -- python3 $R/tools/kernel_probe.py --op $op $kv --iters 5 > $R/gpurun_out/$O/p${i}_$op.log 2>&1 || { echo "pmc $i $op failed"; tail -3 $R/gpurun_out/$O/p${i}_$op.log; exit 1; }
  done
done
cd $R
python tools/pmc_summary.py gpurun_out/$O --match gemm_4w > gpurun_out/$O/summary.md && cat gpurun_out/$O/summary.md
exit 0
