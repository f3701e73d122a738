#!/bin/bash
# r05: the global list's launch order compacted from the row masks (GI_ROW_ORDER=1, default):
# parity suites, then interleaved C2 / C3 A/B against GI_ROW_ORDER=0.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05r
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_configs.py tests/test_gpu_scenes.py tests/test_gpu_features.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -le 1 ] || exit $rc
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], 'global', r['global']['avg_launch_ms'], 'frac', r['frac'], d['image_sha16'])"; }
for v in 1 0 1 0; do
  GI_ROW_ORDER=$v timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$v.log 2>&1 || { tail -5 $D/c2_$v.log; exit 1; }
  line $D/c2_$v.log "c2 rows=$v"
done
for v in 1 0; do
  GI_ROW_ORDER=$v timeout -k 10 300 python3 bench.py --scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --steps 2 --warmup 1 --no-cpu-baseline > $D/c3_$v.log 2>&1 || { tail -5 $D/c3_$v.log; exit 1; }
  line $D/c3_$v.log "c3 rows=$v"
done
exit $rc
