# Round 6: the GPU suite under EDGE_POISON=2 (NaN-filled torch.empty AND all-ones LDS + register files before every
# framework kernel: any read of LDS / VGPR / AGPR a workgroup did not write gives NaN deterministically).
set -o pipefail
O=gpurun_out/${OUT:-r06b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -c "
import torch, llm_inference_in_distributed_edge_networks_amd.ops._native as N
N.lib(); x=torch.zeros(4, device='cuda'); rc=N.lib().edge_poison_lds(N.stream()); torch.cuda.synchronize()
print('poison kernel rc', rc, 'lds bytes', N.lib().edge_poison_lds_bytes())" > $O/probe.log 2>&1 || { cat $O/probe.log; exit 1; }
cat $O/probe.log | grep -v amdgpu.ids
EDGE_POISON=2 timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 40 --timeout 300 --timeout-method thread \
  -p no:cacheprovider -W ignore::UserWarning > $O/pytest_gpu_poison2.log 2>&1
rc=$?
echo "poison2 suite rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O/pytest_gpu_poison2.log | tail -50
exit 0
