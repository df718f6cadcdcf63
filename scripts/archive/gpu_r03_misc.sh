# Round-3 measurements: new GPU tests (graph capture mode, Pythia fp32 relevance), the reference sweep workloads
# (device-side sums + graph-replayed prefix) and BASELINE configs 2-5 through the pipeline entry point (one runtime
# per run, fp32 relevance engine for the head tables).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_lrp_gpu.py tests/test_experiments_gpu.py tests/test_pipeline_gpu.py tests/test_rehearsal_gpu.py -x -q --timeout 300 --timeout-method thread -s -k "pythia or experiments or pipeline or rehearsal or two_ranks or self_launch or four_stage" > gpurun_out/pytest_misc.log 2>&1; rc=$?
echo "[pytest] rc=$rc"; grep -E "passed|failed|pythia-70m normalised" gpurun_out/pytest_misc.log | tail -3; [ $rc -eq 0 ] || exit $rc
TAIL=1 bash scripts/gpu_sweeps.sh || exit $?
bash scripts/gpu_configs.sh || exit $?
exit 0
