set -o pipefail
# round-4: the changed-cell list merge -- GPU suite, then a kernel trace of the cfg3 tick
R=${GRAFT_REPO_ROOT:-$(pwd)}
NO_BENCH=1 bash tools/gpu_run.sh r04o "" || exit 1
bash tools/trace_variants.sh r04o base
