# BASELINE.json configs 2-5 through the Experiments/Pipeline entry point on ONE GPU (stages local, boundary
# messages encoded/decoded as on the wire), synthetic WikiText-2-length stream, random-init weights.
set -o pipefail
mkdir -p gpurun_out/configs
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD_FAIL; tail gpurun_out/build.log; exit 1; }
(cd Experiments/Relevance && timeout -k 10 300 python main.py --max-windows 64 > $R/gpurun_out/configs/relevance.log 2>&1) || { echo RELEVANCE_FAIL; tail $R/gpurun_out/configs/relevance.log; exit 1; }
echo "[relevance] ok"; cp Experiments/Relevance/attention_head_weights.json Experiments/Relevance/channel_group_relevance.json gpurun_out/configs/
cd Experiments/Pipeline
for c in configs/config2_*.json configs/config3_*.json configs/config4_*.json configs/config5_*.json; do
  n=$(basename $c .json)
  case $n in config2*) mw=256;; *) mw=2048;; esac
  timeout -k 10 400 python main.py --params $c --max-windows $mw > $R/gpurun_out/configs/$n.log 2>&1; rc=$?
  echo "[$n] rc=$rc"; grep -v amdgpu $R/gpurun_out/configs/$n.log | grep "ratio=\|pipeline:" ; [ $rc -eq 0 ] || exit $rc
  cp pipeline_results.json $R/gpurun_out/configs/$n.results.json
done
