# rocprofv3 kernel statistics of the fp32 bench (headline config) + h3 GEMM shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 3 --warmup 2 --no-bf16 --no-fp32-weights > $R/gpurun_out/prof.log 2>&1); rc=$?
echo "[prof] rc=$rc"; tail -2 gpurun_out/prof.log
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof -name '*kernel_stats.csv' | head -1); echo "$f"
python tools/prof_summary.py "$f" "bench fp32 N=1" > gpurun_out/prof_summary.md && head -30 gpurun_out/prof_summary.md
timeout -k 10 300 python tools/gemm_bench.py --only h3_gate_up_b64,h3_down_b64,h3_o_proj_b64,h3_qkv_rope_b64,gate_up_b64 --rounds 3 > gpurun_out/gemm.log 2>&1; echo "[gemm] rc=$?"; grep -v "tile=" gpurun_out/gemm.log
exit 0
