set -o pipefail
# round-4 A/B: cell bounds off, tile-order groups, XCD balance, cell-scan cells per thread
bash tools/gpu_variants.sh r04v base nobounds nostayer og4 og8 xcdbal s64i8 s64i4
