set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
ldd llm_inference_in_distributed_edge_networks_amd/_native/libedge_comm.so | grep -i rccl
NCCL_DEBUG=INFO timeout -k 10 180 python tools/rccl_selftest.py > gpurun_out/rccl.log 2>&1; rc=$?
echo "rc=$rc"; grep -v "amdgpu.ids" gpurun_out/rccl.log | tail -40; exit $rc
