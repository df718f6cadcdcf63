set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_e2e.log 2>&1; rc=$?; tail -2 gpurun_out/bench_e2e.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof2.log 2>&1
echo "prof rc=$?"
