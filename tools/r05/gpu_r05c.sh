#!/bin/bash
# r05: MC figure pins + group-kernel parity, then C2 A/B of the large-K group fallback
# (GI_KNN_GROUP / GI_GROUP_CAP), then tools/r05/gpu_r05b.sh (C4 path-kernel A/B, cold frames).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05c
mkdir -p $D
rm -f $D/figs.jsonl
GI_FIG_LOG=$GRAFT_REPO_ROOT/$D/figs.jsonl timeout -k 10 900 python -u -m pytest tests/test_gpu_mc_figs.py "tests/test_gpu_configs.py::test_full_tile_shard_properties" tests/test_gpu_knn_variants.py -k "mc_figure or fresnel or shard or GROUP" -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $D/pytest.log | tail -40
[ $rc -le 1 ] || exit $rc
for g in "1 512" "2 512" "4 512" "4 320" "2 320"; do
  set -- $g
  GI_KNN_GROUP=$1 GI_GROUP_CAP=$2 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_g$1_$2.log 2>&1 || { tail -5 $D/c2_g$1_$2.log; exit 1; }
  grep '^{' $D/c2_g$1_$2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['roofline']['caustic_kernel']; print('group $1 cap $2', d['value'], d['ms_per_step'], 'caustic', c['avg_launch_ms'], 'fallback', c['fallback_avg_ms'], c['fallback_query_frac'], d['image_sha16'])"
done
bash tools/r05/gpu_r05b.sh
exit $rc
