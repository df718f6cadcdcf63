# Round 6: the GPU suite and the multi-rank rehearsal under EDGE_POISON=1 (NaN / 0xFF-filled torch.empty), to expose
# any read of memory nobody wrote for the step (the pp4 rehearsal's intermittent 509.05 vs 503.23).
set -o pipefail
O=gpurun_out/${OUT:-r06a}
mkdir -p $O
export TMPDIR=/tmp
EDGE_POISON=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 40 --timeout 200 --timeout-method thread \
  -p no:cacheprovider -W ignore::UserWarning > $O/pytest_gpu_poison.log 2>&1
rc=$?
echo "poison suite rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $O/pytest_gpu_poison.log | tail -50
[ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
exit 0
