# Round 5: the fp32 QKV epilogue's parts at the bench shape: the production build against probe builds that skip the
# q stores, the K plane stores or the V^T plane stores (build/probe/libedge_kernels_NO_{Q,KP,VP}.so, -DEDGE_PROBE_*
# on a scratch copy of gemm.hip; the macros are not in the committed tree) and the whole epilogue (noepi), interleaved.
set -o pipefail
O=gpurun_out/${OUT:-r05r}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 20 2>/dev/null | sed "s/^/prod  /" >> $O/probe.log || exit 1
  for v in NO_Q NO_KP NO_VP noepi; do
    timeout -k 10 120 env EDGE_KERNEL_LIB=$PWD/build/probe/libedge_kernels_$v.so python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 20 2>/dev/null | sed "s/^/$v /" >> $O/probe.log || exit 1
  done
done
cat $O/probe.log
exit 0
