set -o pipefail
# round-4 final code: the cfg3 profile (kernel trace + PMC passes incl. read-request sizes) and the FETCH calibration
bash tools/profile.sh r04b && bash tools/calib_fetch.sh || exit 1
bash tools/gpu_variants.sh r04r base flatu3 wpe6 qcap512 evw256 ap8 ap2
