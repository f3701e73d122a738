# r06u: the caustic list's 64-bit sort in 10-bit passes (exp/c10: 5 passes instead of 6), and the
# row sort's block shape (exp/rb512: 512 x 16, exp/rb1024x12) against the in-tree library
# (1024 x 16, caustic 8-bit): C2 two rounds, C3 and the C4 shard one round
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06u
mkdir -p $D
: > $D/ab.jsonl
declare -A LIB=([cur]= [c10]=$GRAFT_REPO_ROOT/exp/c10/libgi_amd.so [rb512]=$GRAFT_REPO_ROOT/exp/rb512/libgi_amd.so [rb1024x12]=$GRAFT_REPO_ROOT/exp/rb1024x12/libgi_amd.so)
row() {
  python3 -c "
import json
d=json.loads(open('$1').read().strip().splitlines()[-1])
g=d['roofline']['global']; k=d['roofline']['caustic_kernel']
print(json.dumps({'v':'$2','cfg':'$3','ms':d['ms_per_step'],'g_ms':g['avg_launch_ms'],'c_ms':k['avg_launch_ms'],'sha':d.get('image_sha16')}))" >> $D/ab.jsonl && tail -1 $D/ab.jsonl
}
for r in 1 2; do
  for v in cur c10 rb512 rb1024x12; do
    GI_AMD_LIB=${LIB[$v]} timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2.$v.$r.log 2>&1 || { tail -5 $D/c2.$v.$r.log; exit 1; }
    row $D/c2.$v.$r.log $v c2 || exit 1
  done
done
for v in cur c10; do
  GI_AMD_LIB=${LIB[$v]} timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline > $D/c3.$v.log 2>&1 || { tail -5 $D/c3.$v.log; exit 1; }
  row $D/c3.$v.log $v c3 || exit 1
  GI_AMD_LIB=${LIB[$v]} timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --shard 0/8 --no-cpu-baseline > $D/c4.$v.log 2>&1 || { tail -5 $D/c4.$v.log; exit 1; }
  row $D/c4.$v.log $v c4 || exit 1
done
