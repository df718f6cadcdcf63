# End-to-end A/B of GEMM main-loop choices on one box: bench.py under each EDGE_GEMM_VARIANT in turn.
set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for v in ${VARIANTS:--1 1 -1 1}; do
  EDGE_GEMM_VARIANT=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/ab_$v.log 2>&1 || { tail gpurun_out/ab_$v.log; exit 1; }
  echo "variant $v: $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v.log)"
done
