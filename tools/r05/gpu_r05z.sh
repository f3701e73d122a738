#!/bin/bash
# r05 final tree: smoke(), then the C3 frame, C4 tile shard 0/8 and C5 tile shard 1/8 benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05z
mkdir -p $D
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -5 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
bash tools/r05/gpu_r05o.sh
