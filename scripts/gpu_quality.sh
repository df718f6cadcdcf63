set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 420 python -u tools/train_tiny_lm.py --minutes ${MINUTES:-5} --out gpurun_out/byte_qwen2.safetensors 2>&1 | grep -v amdgpu.ids | tee gpurun_out/train.log; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/quality_sweep.py --windows ${WINDOWS:-1024} > gpurun_out/quality.log 2>&1; rc=$?; echo "[quality] rc=$rc"; grep -v amdgpu.ids gpurun_out/quality.log | head -120
