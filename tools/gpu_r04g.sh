set -o pipefail
# round-4 defaults (no cell bounds, stayer placement, order groups of 8): GPU suite + default bench,
# then kernel traces of the order-group sizes
bash tools/gpu_run.sh r04g "" --steps 20 --warmup 5 || exit 1
bash tools/trace_variants.sh r04g base og1 og4 og16
