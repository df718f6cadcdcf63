# Round 5: sustained throughput (= clock under the power cap at a full pipe) of the 16x16x32 and 32x32x16 fp16 MFMA
# shapes, then one --pmc pass for the per-dispatch clock and MFMA busy.
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
timeout -k 10 120 tools/bin/mfma_power 40 200000 > $O/mfma_power.log 2>&1 || { echo "burn failed"; tail -5 $O/mfma_power.log; exit 1; }
cat $O/mfma_power.log
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d $R/$O/pmc -o run -- $R/tools/bin/mfma_power 20 200000 > $R/$O/pmc.log 2>&1 \
  || { echo "pmc failed"; tail -3 $R/$O/pmc.log; exit 1; }
cd $R
{ python tools/clock_pmc.py $O/pmc "mfma_burnILi0" && python tools/clock_pmc.py $O/pmc "mfma_burnILi1" && python tools/clock_pmc.py $O/pmc "mfma_burnILi2"; } > $O/clock.md
grep -E "median|dispatches" $O/clock.md
exit 0
