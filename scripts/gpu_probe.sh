set -o pipefail
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python tools/determinism_probe3.py > gpurun_out/probe2.log 2>&1; rc=$?
cat gpurun_out/probe2.log | grep -v amdgpu.ids; exit $rc
