set -o pipefail
# round-4 final code: the cfg3 profile (kernel trace + PMC passes incl. read-request sizes) and the FETCH calibration
bash tools/profile.sh r04b && bash tools/calib_fetch.sh
