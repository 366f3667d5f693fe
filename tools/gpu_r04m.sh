set -o pipefail
# round-4: GPU suite + default bench line on the current defaults, then the k_fan_hits A/B
bash tools/gpu_run.sh r04m "" || exit 1
bash tools/gpu_r04l.sh
