# Same-node baseline: the reference's computation on HF transformers + PyTorch eager, fp32, on this MI355X.
set -o pipefail
mkdir -p gpurun_out/hfref
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 420 python -u tools/hf_reference_path_bench.py "$@" > gpurun_out/hfref/$n.json 2> gpurun_out/hfref/$n.err || return $?
  cat gpurun_out/hfref/$n.json
}
run b1_c1 --batch 1 --windows 32 --warmup 2 &&
run b64_c1 --batch 64 --windows 128 --warmup 1 &&
run b1_c100 --batch 1 --windows 2 --warmup 1 --configs 100 &&
run b64_c100 --batch 64 --windows 64 --warmup 1 --configs 100
