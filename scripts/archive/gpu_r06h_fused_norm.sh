# Round 6: RMSNorm-2 fused into the fp32 O-projection epilogue (EPI_F32_RESID_NP).  The new and
# affected fp32 tests, then a same-box A/B of the driver-argument bench (EDGE_FUSED_NORM_F32=0: the separate norm
# pass), interleaved twice, then the kernel profile of the fused step.
set -o pipefail
O=gpurun_out/${OUT:-r06h}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -u -m pytest tests/test_f32_gpu.py -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "np or fused or hidden_state or full_model or four_wave_224 or inplace" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
grep -cE "PASSED" $O/tests.log; grep -E "FAILED|ERROR" $O/tests.log || true
for r in 1 2; do
  for f in 0 1; do
    EDGE_FUSED_NORM_F32=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-bf16 --no-fp32-weights \
      --no-hf-compare --no-sweep --json-out $O/bench_f${f}_$r.json > $O/bench_f${f}_$r.log 2>&1 \
      || { echo "bench f$f failed"; tail -5 $O/bench_f${f}_$r.log; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_f${f}_$r.json')); print('fused=$f run $r', d['value'], d['ms_per_step'], d['ppl_random_weights'], d.get('box_calibration', {}).get('hipblaslt_fp16_tflops'))"
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 --no-bf16 --no-fp32-weights --no-hf-compare --no-sweep > $R/$O/prof.log 2>&1) || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" "fp32 bench step, round 6, RMSNorm-2 fused" > $O/prof_summary.md && head -14 $O/prof_summary.md
exit 0
