#!/bin/bash
# r05: the exact centre bound also in the 1024-candidate second pass (exp/x1024,
# DK_EXACT_MAXCAP=1024) against the in-tree library (first pass only): k-NN parity on x1024,
# then C4 shard and C2 interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05ah
mkdir -p $D
X=$GRAFT_REPO_ROOT/exp/x1024/libgi_amd.so
GI_AMD_LIB=$X timeout -k 10 900 python -u -m pytest tests/test_gpu_knn_variants.py tests/test_gpu_configs.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -le 1 ] || exit $rc
line() { grep '^{' $1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['caustic_kernel']; print('$2', d['value'], d['ms_per_step'], 'caustic', c['avg_launch_ms'], 'p2', c['second_pass_avg_ms'], 'fb', c['fallback_avg_ms'], c['fallback_query_frac'], d['image_sha16'])"; }
for r in 1 2; do
for v in def x1024; do
  L=""; [ $v = x1024 ] && L=$X
  GI_AMD_LIB=$L timeout -k 10 400 python3 bench.py --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8 --steps 1 --warmup 1 > $D/c4.log 2>&1 || { tail -5 $D/c4.log; exit 1; }
  line $D/c4.log "c4 $v $r"
done
done
for v in def x1024; do
  L=""; [ $v = x1024 ] && L=$X
  GI_AMD_LIB=$L timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/c2.log 2>&1 || { tail -5 $D/c2.log; exit 1; }
  line $D/c2.log "c2 $v"
done
exit $rc
