# r06t: (1) the global list's row sort with 30 key bits and no valid count, at 8 (in-tree), 10
# and 11 (exp/r10, exp/r11) radix bits per onesweep pass; (2) no QMETA_NONE stores for the unread
# tiled slots (in-tree; exp/r8ns stores them). Exactness (render + config tests with the in-tree
# library), kernel-trace stats per sort variant, C2 interleaved, C5 shard with and without (2).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06t
mkdir -p $D
: > $D/ab.jsonl
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_render.py tests/test_gpu_configs.py tests/test_gpu_features.py > $D/pytest.log 2>&1 || { tail -20 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
declare -A LIB=([base]=$GRAFT_REPO_ROOT/exp/base/libgi_amd.so [r8]= [r8ns]=$GRAFT_REPO_ROOT/exp/r8ns/libgi_amd.so [r10]=$GRAFT_REPO_ROOT/exp/r10/libgi_amd.so [r11]=$GRAFT_REPO_ROOT/exp/r11/libgi_amd.so)
for v in r8 r10 r11; do
  GI_AMD_LIB=${LIB[$v]} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/$v.prof.log 2>&1 || { tail -20 $D/$v.prof.log; exit 1; }
  echo "$v prof done"
done
row() {
  python3 -c "
import json
d=json.loads(open('$1').read().strip().splitlines()[-1])
g=d['roofline']['global']
print(json.dumps({'v':'$2','cfg':'$3','ms':d['ms_per_step'],'g_ms':g['avg_launch_ms'],'sha':d.get('image_sha16')}))" >> $D/ab.jsonl && tail -1 $D/ab.jsonl
}
for r in 1 2; do
  for v in base r8ns r8 r10 r11; do
    GI_AMD_LIB=${LIB[$v]} timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2.$v.$r.log 2>&1 || { tail -5 $D/c2.$v.$r.log; exit 1; }
    row $D/c2.$v.$r.log $v c2 || exit 1
  done
done
for v in r8ns r8; do
  GI_AMD_LIB=${LIB[$v]} timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 1 --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 0 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8 --no-cpu-baseline > $D/c5.$v.log 2>&1 || { tail -5 $D/c5.$v.log; exit 1; }
  row $D/c5.$v.log $v c5 || exit 1
done
