# Round 5 start: same-box baseline of the fp32 bench step (HEAD) and the clock the chip holds during the two big
# GEMMs (rocprofv3 --kernel-trace + one --pmc pass: SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE against the traced duration).
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
timeout -k 10 180 python -c "import time, __graft_entry__ as g; t=time.time(); g.smoke(); print('smoke s', round(time.time()-t, 1))" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-bf16 --no-fp32-weights --no-hf-compare \
  --json-out $O/bench.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'])"
cd /tmp
for op in gateup down; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_MFMA \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $R/$O/clk_$op -o run -- \
    python3 $R/tools/kernel_probe.py --op $op --iters 4 > $R/$O/clk_$op.log 2>&1 \
    || { echo "pmc $op failed"; tail -3 $R/$O/clk_$op.log; exit 1; }
done
cd $R
python tools/clock_pmc.py $O/clk_gateup "gemm_4w_kernel<13" > $O/clock.md && python tools/clock_pmc.py $O/clk_down "gemm_4w_kernel<10" >> $O/clock.md && cat $O/clock.md
exit 0
