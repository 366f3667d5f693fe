set -o pipefail
# round-4: GPU suite + default bench line on the current code, then the two-phase finish and the
# fixup-in-keygen A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
bash tools/gpu_run.sh r04n "" || exit 1
bash tools/gpu_variants.sh r04n base fin2 fixkg
