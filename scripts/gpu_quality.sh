set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
# outputs go straight to files under gpurun_out/ (a pipe through grep/tee would hold them back)
timeout -k 10 480 python -u tools/train_tiny_lm.py --minutes ${MINUTES:-5} --out /tmp/byte_qwen2.safetensors > gpurun_out/train.log 2>&1; rc=$?
echo "[train] rc=$rc"; tail -4 gpurun_out/train.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/quality_sweep.py --windows ${WINDOWS:-1024} > gpurun_out/quality.log 2>&1; rc=$?
echo "[quality] rc=$rc"; grep -c "|" gpurun_out/quality.log; exit $rc
