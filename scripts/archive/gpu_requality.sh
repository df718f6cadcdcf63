# Re-measure after the constant-mask fix: configs 3-5 quality (trained byte-Qwen2) and configs 2-5 entry points.
set -o pipefail
bash scripts/gpu_pipeline_quality.sh || exit $?
bash scripts/gpu_configs.sh || exit $?
exit 0
