# PMC counters of the GEMM variants (rocprofv3 --pmc, kernel counters only; no trace domains).
# env: TILES (gemm_bench --tiles), SHAPES, OUT (dir under gpurun_out)
set -o pipefail
OUT=${OUT:-pmc3}
mkdir -p gpurun_out/$OUT
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
cd /tmp
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$OUT/$tag -o run -- python $GRAFT_REPO_ROOT/tools/gemm_bench.py --only ${SHAPES:-gate_up_b64,down_b64} --rounds 1 --iters 3 --tiles ${TILES:-256} --no-lib > $GRAFT_REPO_ROOT/gpurun_out/$OUT/$tag.log 2>&1 || { echo "pmc $tag failed"; tail $GRAFT_REPO_ROOT/gpurun_out/$OUT/$tag.log; exit 1; }
done
echo pmc done
