# Quality sweep on a byte-level Qwen2 trained on the box (no checkpoints are reachable): PPL vs boundary codec,
# fp32 and bf16 execution.  env: MINUTES (training), WINDOWS, CODECS, DTYPES
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
# outputs go straight to files under gpurun_out/ (a pipe through grep/tee would hold them back); the weights stay in
# /tmp (gpurun_out is size-capped)
timeout -k 10 480 python -u tools/train_tiny_lm.py --minutes ${MINUTES:-5} --out /tmp/byte_qwen2.safetensors > gpurun_out/train.log 2>&1; rc=$?
echo "[train] rc=$rc"; tail -4 gpurun_out/train.log; [ $rc -eq 0 ] || exit $rc
CODECS=${CODECS:-ref_int4_global,int4_token,mixed_int4_int8,mixed_int2_int8,mxfp4,mxfp8,mixed_mxfp4_mxfp8,mxfp4_keep}
for dt in ${DTYPES:-fp32 bf16}; do
  timeout -k 10 600 python -u tools/quality_sweep.py --windows ${WINDOWS:-1024} --dtype $dt --codecs $CODECS \
    --json-out gpurun_out/quality_sweep_$dt.json > gpurun_out/quality_$dt.log 2>&1; rc=$?
  echo "[quality $dt] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
