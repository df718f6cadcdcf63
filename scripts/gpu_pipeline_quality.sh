# BASELINE configs 3-5 through the real multi-boundary pipeline on a byte-level Qwen2 trained on the box (no
# checkpoint is reachable): PPL vs wire bytes at 1, 3 and 7 quantized boundaries.  env: MINUTES, WINDOWS
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 480 python -u tools/train_tiny_lm.py --minutes ${MINUTES:-5} --out /tmp/byte_qwen2.safetensors > gpurun_out/train.log 2>&1; rc=$?
echo "[train] rc=$rc"; tail -3 gpurun_out/train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/pipeline_quality.py --windows ${WINDOWS:-1024} \
  --json-out gpurun_out/pipeline_quality.json > gpurun_out/pipeline_quality.log 2>&1; rc=$?
echo "[pipeline_quality] rc=$rc"; tail -30 gpurun_out/pipeline_quality.log; [ $rc -eq 0 ] || exit $rc
exit 0
