#!/bin/bash
# FETCH_SIZE calibration for k_combined's read shapes (tools/calib_fetch.hip), on the GPU box.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/calib_fetch
mkdir -p $OUT
# built here, not tracked (hipcc is on the box too)
[ -x $R/goworld_amd/lib/calib_fetch ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o $R/goworld_amd/lib/calib_fetch $R/tools/calib_fetch.hip
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $R/goworld_amd/lib/calib_fetch > $OUT/calib.json 2> $OUT/fetch.err
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d $OUT/rdreq -o run -- $R/goworld_amd/lib/calib_fetch > /dev/null 2> $OUT/rdreq.err
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- $R/goworld_amd/lib/calib_fetch > /dev/null 2> $OUT/trace.err
ls -R $OUT | head
