#!/bin/bash
# r05: lane-select and launch-order variants (exp/<v>/libgi_amd.so vs the in-tree library "hil"):
# k-NN parity on the in-tree library, then interleaved C2 benches (global k-NN per launch, frame).
#   base: r05 tree; p: phased packed d2 (no s_nop); pad: p + the bracket sorted by a Batcher
#   network sized to the wave (4 / 8 / 12 keys); hil: pad + Hilbert-curve launch order
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r05m
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_knn_variants.py tests/test_gpu_render.py tests/test_gpu_configs.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $D/pytest.log 2>&1
rc=$?
tail -3 $D/pytest.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for v in base p pad hil; do
    L=""; [ $v != hil ] && L=$GRAFT_REPO_ROOT/exp/$v/libgi_amd.so
    GI_AMD_LIB=$L timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$v.$r.log 2>&1 || { tail -5 $D/c2_$v.$r.log; exit 1; }
    grep '^{' $D/c2_$v.$r.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c2 $v $r', d['value'], d['ms_per_step'], 'global', r['global']['avg_launch_ms'], 'frac', r['frac'], d['image_sha16'])"
  done
done
exit $rc
