#!/bin/bash
# A/B of libgwaoi build variants on the cfg3 tick: parity subset per variant, then one kernel trace each.
# usage: bash tools/gpu_variants.sh TAG NAME...   (NAME = goworld_amd/lib/variants/NAME.so; base = default lib)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for v in "$@"; do
  [ "$v" = base ] && continue
  GWAOI_LIB=$R/goworld_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread -k "scaled_configs or speculative or incremental_sort or repeated or device_batch or zero_copy" > $R/gpurun_out/pytest_${TAG}_$v.log 2>&1 || { echo "parity $v failed"; tail -20 $R/gpurun_out/pytest_${TAG}_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $R/gpurun_out/pytest_${TAG}_$v.log)"
done
bash $R/tools/trace_variants.sh $TAG "$@"
