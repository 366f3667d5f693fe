set -o pipefail
# round-4 profile: kernel trace + PMC passes of the cfg3 tick, then the FETCH_SIZE calibration
bash tools/profile.sh r04 && bash tools/calib_fetch.sh
