set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python tools/gemm_bench.py --rounds 3 --iters 10 --tiles ${TILES:-256,256s,256s-a1,256s-a3} --only gate_up_b64,down_b64,big --no-lib > gpurun_out/abl.log 2>&1; rc=$?
grep -v amdgpu gpurun_out/abl.log; exit $rc
