#!/bin/bash
# r05: large-K chunk pass chain A/B (GI_CHUNK_CAP_BIG2/3): exactness, then C4 shard 0/8, C3, C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05g
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_knn_variants.py -k "CAP_BIG or rim" -q -x -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -eq 0 ] || exit $rc
C4="--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --shard 0/8"
C3="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000"
run() {  # name env... : C4 shard, C3, C2 lines
  n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py $C4 --steps 2 --warmup 1 --no-cpu-baseline > $D/c4_$n.log 2>&1 || { tail -5 $D/c4_$n.log; return 1; }
  grep '^{' $D/c4_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['caustic_kernel']; print('c4 $n', d['ms_per_step'], 'caustic', c['avg_launch_ms'], 'p2', c['second_pass_avg_ms'], c['second_pass_query_frac'], 'fb', c['fallback_avg_ms'], c['fallback_query_frac'])"
  env "$@" timeout -k 10 300 python3 bench.py $C3 --steps 2 --warmup 1 --no-cpu-baseline > $D/c3_$n.log 2>&1 || { tail -5 $D/c3_$n.log; return 1; }
  grep '^{' $D/c3_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['caustic_kernel']; print('c3 $n', d['ms_per_step'], 'caustic', c['avg_launch_ms'], 'p2', c['second_pass_avg_ms'], 'fb', c['fallback_avg_ms'], d['image_sha16'])"
  env "$@" timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$n.log 2>&1 || { tail -5 $D/c2_$n.log; return 1; }
  grep '^{' $D/c2_$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['caustic_kernel']; print('c2 $n', d['ms_per_step'], 'caustic', c['avg_launch_ms'], 'p2', c['second_pass_avg_ms'], 'fb', c['fallback_avg_ms'], d['image_sha16'])"
}
run base GI_NONE=0 || exit 1
run c576 GI_CHUNK_CAP_BIG2=576 || exit 1
run c576_1024 GI_CHUNK_CAP_BIG2=576 GI_CHUNK_CAP_BIG3=1024 || exit 1
run base2 GI_NONE=0 || exit 1
