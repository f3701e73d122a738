#!/bin/bash
# r05: the large-K chunk kernel's centre bound refined to the exact d_K(c) (GI_CHUNK_DK_EXACT=1):
# k-NN / render / config parity with it on, then C2, C3 and the C4 shard with it off / on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05ag
mkdir -p $D
GI_CHUNK_DK_EXACT=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_knn_variants.py tests/test_gpu_render.py tests/test_gpu_configs.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -le 1 ] || exit $rc
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['caustic_kernel']; print('$2', d['value'], d['ms_per_step'], 'caustic', c['avg_launch_ms'], 'p2', c['second_pass_avg_ms'], c['second_pass_query_frac'], 'fb', c['fallback_avg_ms'], c['fallback_query_frac'], 'vis', round(c['visited_per_query'],1), d['image_sha16'])"; }
for v in 0 1; do
  GI_CHUNK_DK_EXACT=$v timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/c2.log 2>&1 || { tail -5 $D/c2.log; exit 1; }
  line $D/c2.log "c2 exact=$v"
  GI_CHUNK_DK_EXACT=$v timeout -k 10 300 python3 bench.py --scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --steps 2 --warmup 1 --no-cpu-baseline > $D/c3.log 2>&1 || { tail -5 $D/c3.log; exit 1; }
  line $D/c3.log "c3 exact=$v"
  GI_CHUNK_DK_EXACT=$v timeout -k 10 400 python3 bench.py --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8 --steps 1 --warmup 1 > $D/c4.log 2>&1 || { tail -5 $D/c4.log; exit 1; }
  line $D/c4.log "c4 exact=$v"
done
exit $rc
