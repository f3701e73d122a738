#!/bin/bash
# r05: lane-select one-store collect (LS_ONE_STORE) exactness + C2 A/B; cold first frames of
# C5 shard 1/8 and C2 with the allocation log (call sites) and the Monte Carlo append sizing.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05d
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_knn_variants.py "tests/test_gpu_render.py::test_c2_config_matches_oracle" tests/test_gpu_configs.py -k "not GROUP and not full" -q -x -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -eq 0 ] || exit $rc
for l in exp/ls0/libgi_amd.so default exp/ls0/libgi_amd.so default; do
  if [ $l = default ]; then unset GI_AMD_LIB; n=ls1; else export GI_AMD_LIB=$l; n=ls0; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $D/c2_$n.log 2>&1 || { tail -5 $D/c2_$n.log; exit 1; }
  grep '^{' $D/c2_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['roofline']['global']; print('$n', d['value'], d['ms_per_step'], 'global knn', g['avg_launch_ms'], 'frac', d['roofline']['frac'], 'first', d['first_frame_ms'], d['image_sha16'])"
done
unset GI_AMD_LIB
C5="--scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 1 --shard 1/8"
GI_BATCH_LOG=1 GI_ALLOC_LOG=1 timeout -k 10 400 python3 bench.py $C5 "--extra=-dof 4 12.2282 0.025 -no_caustic" --steps 1 --warmup 1 --no-cpu-baseline > $D/c5_cold.log 2>&1 || { tail -5 $D/c5_cold.log; exit 1; }
grep '^{' $D/c5_cold.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 shard1/8', d['ms_per_step'], 'first', d['first_frame_ms'])"
grep -E "alloc.*: [0-9]{3,}\.[0-9] ms" $D/c5_cold.log | head
GI_BATCH_LOG=1 GI_ALLOC_LOG=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/c2_cold.log 2>&1 || { tail -5 $D/c2_cold.log; exit 1; }
grep '^{' $D/c2_cold.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 cold', d['value'], d['ms_per_step'], 'first', d['first_frame_ms'], d['image_sha16'])"
grep "path passes 2" $D/c2_cold.log | head -3
exit 0
