# Round 4: PMC passes (kernel counters only, no trace domains) over the fp32 AttnLRP engine at 64 windows: the x6
# attention backward (dK/dV, dQ), the fused SwiGLU + pre-activation GEMM, the SwiGLU rule, the vector RoPE pack.
# Summary: tools/pmc_kernels.py.
set -o pipefail
OUT=r04p_pmc
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/$OUT/p$i -o run -- python3 $R/tools/relevance_bench.py --dtype fp32 --batch 64 --iters 1 --warmup 0 > $R/gpurun_out/$OUT/p$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $R/gpurun_out/$OUT/p$i.log; exit 1; }
done
cd $R
python tools/pmc_kernels.py gpurun_out/$OUT lrp_attn_dkdv_x6 lrp_attn_dq_x6 "gemm_4w_kernel<13" lrp_swiglu_bwd_h3 lrp_rope_pack_h3_v4 "gemm_4w_kernel<16" > gpurun_out/$OUT/summary.md && cat gpurun_out/$OUT/summary.md
exit 0
