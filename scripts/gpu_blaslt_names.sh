set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_gemm -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/gemm_bench.py --rounds 1 --iters 5 --only gate_up_b64,down_b64,o_proj_b64,qkv > $GRAFT_REPO_ROOT/gpurun_out/prof_gemm.log 2>&1
echo "[prof] rc=$?"; tail -8 $GRAFT_REPO_ROOT/gpurun_out/prof_gemm.log
