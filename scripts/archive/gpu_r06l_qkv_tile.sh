set -o pipefail
mkdir -p gpurun_out/r06l
for r in 1 2 3; do
  for t in 0 256; do
    timeout -k 10 120 python tools/kernel_probe.py --op qkv --kv-planes 1 --iters 40 --tile $t > gpurun_out/r06l/qkv_t${t}_$r.log 2>&1 || { echo "probe failed"; tail -5 gpurun_out/r06l/qkv_t${t}_$r.log; exit 1; }
    echo "tile $t run $r: $(tail -1 gpurun_out/r06l/qkv_t${t}_$r.log)"
  done
done
for t in 0 256; do timeout -k 10 120 python tools/kernel_probe.py --op gateup --iters 20 --tile $t > gpurun_out/r06l/gateup_t$t.log 2>&1; echo "gateup tile $t: $(tail -1 gpurun_out/r06l/gateup_t$t.log)"; done
