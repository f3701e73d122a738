#!/bin/bash
# r05: early k-NN of the deterministic query slots before the Monte Carlo join (GI_EARLY_KNN):
# the parity suites, then interleaved C2 / C3 A/B against GI_EARLY_KNN=0.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05k
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_configs.py tests/test_gpu_scenes.py tests/test_gpu_features.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -5 $D/pytest.log
[ $rc -le 1 ] || exit $rc
C3="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000"
for v in 1 0 1 0; do
  GI_EARLY_KNN=$v timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$v.log 2>&1 || { tail -5 $D/c2_$v.log; exit 1; }
  grep '^{' $D/c2_$v.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2 early=$v', d['value'], d['ms_per_step'], 'first', d['first_frame_ms'], 'global', r['global']['avg_launch_ms'], 'frac', r['frac'], 'caustic', r['caustic_kernel']['avg_launch_ms'], d['image_sha16'])"
done
for v in 1 0; do
  GI_EARLY_KNN=$v timeout -k 10 300 python3 bench.py $C3 --steps 2 --warmup 1 --no-cpu-baseline > $D/c3_$v.log 2>&1 || { tail -5 $D/c3_$v.log; exit 1; }
  grep '^{' $D/c3_$v.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 early=$v', d['value'], d['ms_per_step'], d['image_sha16'])"
done
exit $rc
