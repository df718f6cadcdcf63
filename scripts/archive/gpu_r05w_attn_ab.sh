# Round 5: attention forward A/B (HEAD build vs the product-major MFMA order), longer runs: 200 calls per process,
# 4 interleaved rounds.
set -o pipefail
O=gpurun_out/${OUT:-r05w}
mkdir -p $O
HEAD_LIB=$PWD/build/ab_attn/libedge_kernels_head.so
for r in 1 2 3 4; do
  timeout -k 10 120 env EDGE_KERNEL_LIB=$HEAD_LIB python tools/kernel_probe.py --op attn --kv-planes 1 --iters 200 2>/dev/null | sed "s/^/head /" >> $O/probe.log || exit 1
  timeout -k 10 120 python tools/kernel_probe.py --op attn --kv-planes 1 --iters 200 2>/dev/null | sed "s/^/new  /" >> $O/probe.log || exit 1
done
cat $O/probe.log
exit 0
