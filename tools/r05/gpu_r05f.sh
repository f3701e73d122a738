#!/bin/bash
# r05: ray_tri's division-free rejection (RAY_TRI_PRETEST): the image-parity suites, then
# interleaved A/B against exp/pre0 on C2, C4 shard 0/8 and C5 shard 1/8.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05f
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_scenes.py tests/test_gpu_render.py tests/test_gpu_features.py tests/test_gpu_configs.py -q -x -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -eq 0 ] || exit $rc
C4="--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --shard 0/8"
C5="--scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1 --shard 1/8"
for l in default exp/pre0/libgi_amd.so default exp/pre0/libgi_amd.so; do
  if [ $l = default ]; then unset GI_AMD_LIB; n=pre1; else export GI_AMD_LIB=$l; n=pre0; fi
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$n.log 2>&1 || { tail -5 $D/c2_$n.log; exit 1; }
  grep '^{' $D/c2_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 $n', d['value'], d['ms_per_step'], d['image_sha16'])"
done
for l in default exp/pre0/libgi_amd.so; do
  if [ $l = default ]; then unset GI_AMD_LIB; n=pre1; else export GI_AMD_LIB=$l; n=pre0; fi
  timeout -k 10 300 python3 bench.py $C4 --steps 2 --warmup 1 --no-cpu-baseline > $D/c4_$n.log 2>&1 || { tail -5 $D/c4_$n.log; exit 1; }
  grep '^{' $D/c4_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4 $n', d['value'], d['ms_per_step'], d['step_ms'])"
  timeout -k 10 400 python3 bench.py $C5 "--extra=-dof 4 12.2282 0.025 -no_caustic" --steps 1 --warmup 1 --no-cpu-baseline > $D/c5_$n.log 2>&1 || { tail -5 $D/c5_$n.log; exit 1; }
  grep '^{' $D/c5_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 $n', d['value'], d['ms_per_step'])"
done
