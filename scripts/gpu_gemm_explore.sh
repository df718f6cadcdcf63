set -o pipefail
mkdir -p gpurun_out
EDGE_TUNING=1 EDGE_KERNEL_LIB=$PWD/build/tuning/libedge_kernels.so timeout -k 10 500 python tools/gemm_bench.py --only h3_2t_gate_up_b64,h3_2t_down_b64 --tiles 0,0/nob1,0/nob,0/noepi --rounds 3 > gpurun_out/gemm_explore.log 2>&1; rc=$?
echo "[gemm] rc=$rc"; cat gpurun_out/gemm_explore.log | grep -v amdgpu.ids
exit $rc
