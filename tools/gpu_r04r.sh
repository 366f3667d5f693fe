set -o pipefail
# round-4 retune at D/3 cells: flat-sweep chunks per iteration, waves per SIMD, queue / event buffer sizes,
# moves per apply thread
bash tools/gpu_variants.sh r04r base flatu3 wpe6 qcap512 evw256 ap8 ap2
