# Round 6: more 4-rank pp4 repeats of the round-5 one-off, bit-compared window by window with the single process:
# 12 with a fifth process flooding the GPU, then 12 under EDGE_POISON=2 (uninitialised reads give NaN every time).
set -o pipefail
O=gpurun_out/${OUT:-r06m}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/rehearsal_stress.py --runs 12 --hog-seconds 400 --out $O/hog > $O/hog.log 2>&1 \
  || { echo "hog stress rc=$?"; tail -5 $O/hog.log; exit 1; }
tail -1 $O/hog.log | cut -c1-300
EDGE_POISON=2 timeout -k 10 500 python -u tools/rehearsal_stress.py --runs 12 --out $O/poison > $O/poison.log 2>&1 \
  || { echo "poison stress rc=$?"; tail -5 $O/poison.log; exit 1; }
tail -1 $O/poison.log | cut -c1-300
exit 0
