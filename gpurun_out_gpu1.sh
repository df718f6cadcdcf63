set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; cat gpurun_out/build.log | tail; exit 1; }
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench1.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
echo "prof rc=$?"
