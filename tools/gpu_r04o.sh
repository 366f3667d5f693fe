set -o pipefail
# round-4: the changed-cell list merge and the key aliasing -- GPU suite; then the two-phase finish A/B
R=${GRAFT_REPO_ROOT:-$(pwd)}
NO_BENCH=1 bash tools/gpu_run.sh r04o "" || exit 1
bash tools/gpu_variants.sh r04o base fin2
