# Round 5: how much of the fp32 QKV GEMM (256x192 tiles, bench shape) is its epilogue: the production build against a
# probe build whose QKV epilogue returns before any load or store (build/probe/libedge_kernels_noepi.so, built with
# -DEDGE_PROBE_QKV_NOEPI from the same sources; the macro is not in the committed tree), interleaved.
set -o pipefail
O=gpurun_out/${OUT:-r05q}
mkdir -p $O
NOEPI=$PWD/build/probe/libedge_kernels_noepi.so
for r in 1 2 3; do
  timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 20 2>/dev/null | sed "s/^/prod  /" >> $O/probe.log || exit 1
  timeout -k 10 120 env EDGE_KERNEL_LIB=$NOEPI python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 20 2>/dev/null | sed "s/^/noepi /" >> $O/probe.log || exit 1
done
for r in 1 2; do
  timeout -k 10 120 python tools/kernel_probe.py --op attn --kv-planes 1 --iters 20 2>/dev/null | sed "s/^/attn  /" >> $O/probe.log || exit 1
  timeout -k 10 120 python tools/kernel_probe.py --op norm --iters 20 2>/dev/null | sed "s/^/norm  /" >> $O/probe.log || exit 1
done
cat $O/probe.log
exit 0
