# Round 4 re-entry (rebuilt container), one box: the full GPU check (suite, smoke, bench with the driver's arguments,
# fp32 / bf16 AttnLRP at 64 windows), then the kernel profiles of the fp32 bench step and the fp32 AttnLRP engine.
set -o pipefail
bash scripts/gpu_r04z5_check.sh || exit 1
bash scripts/gpu_r04z6_prof.sh || exit 1
exit 0
