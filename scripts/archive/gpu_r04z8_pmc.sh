# Round 4 end: PMC passes (kernel counters only, no trace domains) over the fp32 bench step's two largest GEMMs
# (gate/up + SwiGLU h3 planes, down + fp32 residual) at the bench shape, current build: MFMA busy per SIMD cycle,
# wait share, VALU per MFMA, LDS bank conflicts.  Summary: tools/pmc_kernels.py.
set -o pipefail
OUT=r04z8_pmc
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for op in gateup down; do
  timeout -k 10 120 python tools/kernel_probe.py --op $op --iters 5 > gpurun_out/$OUT/time_$op.log 2>&1 || { echo "time $op failed"; tail gpurun_out/$OUT/time_$op.log; exit 1; }
  tail -1 gpurun_out/$OUT/time_$op.log
done
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for op in gateup down; do
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/$OUT/p${i}/$op -o run -- python3 $R/tools/kernel_probe.py --op $op --iters 3 > $R/gpurun_out/$OUT/p${i}_$op.log 2>&1 || { echo "pmc $i $op failed"; tail -3 $R/gpurun_out/$OUT/p${i}_$op.log; exit 1; }
  done
done
cd $R
python tools/pmc_kernels.py gpurun_out/$OUT "gemm_4w_kernel<13" "gemm_4w_kernel<10" > gpurun_out/$OUT/summary.md && cat gpurun_out/$OUT/summary.md
exit 0
