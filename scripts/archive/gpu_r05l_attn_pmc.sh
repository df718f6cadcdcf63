# Round 5: clock and MFMA-pipe occupancy of the fp32 attention (plane-staged) and the QKV GEMM at the bench shape.
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
cd /tmp
for op in attn qkv; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_MFMA \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAIT_INST_ANY --output-format csv -d $R/$O/clk_$op -o run -- \
    python3 $R/tools/kernel_probe.py --op $op --kv-planes 1 --iters 12 > $R/$O/clk_$op.log 2>&1 \
    || { echo "pmc $op failed"; tail -3 $R/$O/clk_$op.log; exit 1; }
done
cd $R
{ python tools/clock_pmc.py $O/clk_attn "flash_attn_fwd_x6" && python tools/clock_pmc.py $O/clk_qkv "gemm_4w_kernel<14"; } > $O/clock.md
grep -E "median|dispatches" $O/clock.md
python - <<'PY'
import csv, glob, collections
for op in ("attn", "qkv"):
    tot = collections.Counter(); n = 0
    for f in glob.glob(f"gpurun_out/r05l/clk_{op}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if ("flash_attn_fwd_x6" if op == "attn" else "gemm_4w_kernel<14") in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    if tot:
        print(op, "VALU/MFMA %.2f" % (tot["SQ_INSTS_VALU"] / max(tot["SQ_INSTS_MFMA"], 1)),
              "wait_any/wave %.3f" % (tot["SQ_WAIT_ANY"] / max(tot["SQ_WAVE_CYCLES"], 1)),
              "wait_inst/wave %.3f" % (tot["SQ_WAIT_INST_ANY"] / max(tot["SQ_WAVE_CYCLES"], 1)))
PY
exit 0
