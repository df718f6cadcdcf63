# Round 6: the 24-layer Qwen2-0.5B-shape byte surrogate trained with a fixed start-of-window token
# (--bos 256, the position Qwen2's sink sits at) for ~2.3x round 5's budget, logging the boundary tensors' peak / RMS at
# the notebook layers (3, 11, 18, 22, 23) at every evaluation; then, in the same call (the checkpoint cannot be pulled
# back), the notebook sweep with the three findings (Q1, bootstrap intervals) and configs 3-5 through the pipeline
# with the MSE-allocated head-group plans, all on BOS windows.
set -o pipefail
O=gpurun_out/${OUT:-r06d}
mkdir -p $O
export TMPDIR=/tmp
W=/tmp/byte_qwen2_24_bos.safetensors
timeout -k 10 ${TRAIN_TO:-780} python -u tools/train_tiny_lm.py --model byte-qwen2-24 --out $W --minutes ${TRAIN_MIN:-10.5} \
  --seed ${SEED:-0} --lr ${LR:-1e-3} --warmup 200 --batch 64 --seq 512 --eval-every 30 --patience 1000 --bos 256 --weight-decay ${WD:-0.1} \
  > $O/train.log 2>&1 || { echo "train failed"; tail -20 $O/train.log; exit 1; }
grep probe_step $O/train.log | tail -4 | cut -c1-400
tail -2 $O/train.log | cut -c1-600
if [ "${SKIP_SWEEP:-0}" != 1 ]; then
timeout -k 10 330 python -u tools/quality_sweep.py --model byte-qwen2-24 --weights $W --layers 22,18,3,23,11 --bos 256 \
  --codecs ${CODECS:-ref_int4_global,int4_token,mixed_int4_int8,mixed_rgroup_int8@4,mixed_rgroup_int8@4u} \
  --windows ${WINDOWS:-1024} --batch 16 --boot 1000 --json-out $O/quality_sweep.json > $O/quality_sweep.log 2>&1 \
  || { echo "sweep failed"; tail -20 $O/quality_sweep.log; exit 1; }
grep -E "^###|relevance:|outliers|plans|hurts|column-mean -|ratio 1 -" $O/quality_sweep.log | head -60 || true
fi
[ "${SKIP_PIPE:-0}" = 1 ] && exit 0
timeout -k 10 270 python -u tools/pipeline_quality.py --model byte-qwen2-24 --weights $W --splits bench --bos 256 \
  --windows ${WINDOWS:-1024} --json-out $O/pipeline_quality.json > $O/pipeline_quality.log 2>&1 \
  || { echo "pipeline quality failed"; tail -20 $O/pipeline_quality.log; exit 1; }
tail -32 $O/pipeline_quality.log
exit 0
