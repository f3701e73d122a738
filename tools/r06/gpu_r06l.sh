# r06l: C5 cold first frame (fresh box, first process) with growth capped at 1.5x the request;
# then the second chunk pass's sub-chunk floor (GI_CHUNK_MINSUB2) on the C5 shard and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06l
mkdir -p $D
: > $D/ab.jsonl
C5=(--scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 0 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8)
row() {  # row <log> <tag>
  python3 -c "
import json
d=json.loads(open('$1').read().strip().splitlines()[-1])
g=d['roofline']['global']
print(json.dumps({'tag':'$2','ms':d['ms_per_step'],'first':d.get('first_frame_ms'),'steps':d.get('step_ms'),'global':g,'sha':d.get('image_sha16')}))" >> $D/ab.jsonl && tail -1 $D/ab.jsonl
}
GI_LOG=1 timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 "${C5[@]}" --no-cpu-baseline > $D/c5.cold.log 2>&1 || { tail -5 $D/c5.cold.log; exit 1; }
row $D/c5.cold.log c5.cold || exit 1
for v in 16 8 4 32; do
  GI_CHUNK_MINSUB2=$v timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 1 "${C5[@]}" --no-cpu-baseline > $D/c5.m$v.log 2>&1 || { tail -5 $D/c5.m$v.log; exit 1; }
  row $D/c5.m$v.log c5.minsub2=$v || exit 1
done
GI_CHUNK_MINSUB=16 GI_CHUNK_MINSUB2=8 timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 1 "${C5[@]}" --no-cpu-baseline > $D/c5.m16_8.log 2>&1 || { tail -5 $D/c5.m16_8.log; exit 1; }
row $D/c5.m16_8.log c5.minsub=16,minsub2=8 || exit 1
for v in 32 8 16 32 8; do
  GI_CHUNK_MINSUB2=$v timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2.m$v.log 2>&1 || { tail -5 $D/c2.m$v.log; exit 1; }
  row $D/c2.m$v.log c2.minsub2=$v || exit 1
done
