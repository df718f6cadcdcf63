# Round 5: quality surrogate with statistics.  SEED=n.  Train the 24-layer Qwen2-0.5B-shape byte
# model on the large local corpus with a held-out-driven stop, then in the same call (the checkpoint cannot be pulled
# back): the notebook sweep with per-window bootstrap intervals and the three findings, and configs 3-5 through the
# multi-boundary pipeline with the sensitivity (MSE) / relevance / uniform head-group plans at 4 and 3 bits.
# TESTS=1: first the GPU tests of the codec and LRP kernels this run depends on.
set -o pipefail
O=gpurun_out/r05c_s${SEED:-0}
mkdir -p $O
export TMPDIR=/tmp
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_lrp_gpu.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider -k "group or codec or absprod or engine_h3_tiny or helpers or rule" \
    > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
W=/tmp/byte_qwen2_24.safetensors
timeout -k 10 420 python -u tools/train_tiny_lm.py --model byte-qwen2-24 --out $W --minutes ${TRAIN_MIN:-4.5} \
  --seed ${SEED:-0} --lr 6e-4 --warmup 100 --batch 64 --seq 512 --eval-every 20 --patience 4 \
  > $O/train.log 2>&1 || { echo "train failed"; tail -20 $O/train.log; exit 1; }
tail -2 $O/train.log
timeout -k 10 420 python -u tools/quality_sweep.py --model byte-qwen2-24 --weights $W --layers 22,18,3,23,11 \
  --codecs ref_int4_global,mixed_int4_int8,mixed_rgroup_int8@4,mixed_rgroup_int8@4r,mixed_rgroup_int8@4u,mixed_rgroup_int8@3,mixed_rgroup_int8@3u \
  --windows ${WINDOWS:-2048} --batch 16 --boot 1000 --json-out $O/quality_sweep.json > $O/quality_sweep.log 2>&1 \
  || { echo "sweep failed"; tail -20 $O/quality_sweep.log; exit 1; }
grep -E "^###|relevance:|plans|findings|hurts|column-mean -|ratio 1 -" $O/quality_sweep.log | head -60 || true
timeout -k 10 360 python -u tools/pipeline_quality.py --model byte-qwen2-24 --weights $W --splits bench \
  --windows ${WINDOWS:-2048} --json-out $O/pipeline_quality.json > $O/pipeline_quality.log 2>&1 \
  || { echo "pipeline quality failed"; tail -20 $O/pipeline_quality.log; exit 1; }
tail -32 $O/pipeline_quality.log
exit 0
