# r06 interleaved A/B: exp/base/libgi_amd.so (GI_AMD_LIB) against the in-tree library on C2, C3
# and the C4 tile shard 0/8 -- or, with VAR="NAME=value", the in-tree library with and without
# that environment knob; one JSON line per run (frame ms, global / caustic k-NN ms per launch,
# image hash) into gpurun_out/$OUT/ab.jsonl.
# usage: OUT=r06e ROUNDS=2 CFGS="c2 c3 c4" [VAR=GI_MC_PERSIST=1] bash tools/r06/ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUT:-ab}
mkdir -p $D
: > $D/ab.jsonl
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in base new; do
    L=""; E=()
    if [ -n "$VAR" ]; then [ $v = new ] && E=("$VAR")
    elif [ $v = base ]; then L=$GRAFT_REPO_ROOT/exp/base/libgi_amd.so; fi
    for c in ${CFGS:-c2 c3}; do
      case $c in
        c2) A=(--steps 3 --warmup 1);;
        c3) A=(--steps 2 --warmup 1 --scene jensen.scn --global-photons 2176 --caustic-photons 4000000);;
        c4) A=(--steps 2 --warmup 1 --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --shard 0/8);;
        c5) A=(--steps 1 --warmup 1 --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 0 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8);;
      esac
      env "${E[@]}" GI_AMD_LIB=$L timeout -k 10 400 python3 -u bench.py "${A[@]}" --no-cpu-baseline > $D/$c.$v.$r.log 2>&1 || { tail -5 $D/$c.$v.$r.log; exit 1; }
      python3 -c "
import json
d=json.loads(open('$D/$c.$v.$r.log').read().strip().splitlines()[-1])
g=d['roofline']['global']; k=d['roofline']['caustic_kernel']
print(json.dumps({'cfg':'$c','v':'$v','round':$r,'ms':d['ms_per_step'],'first':d.get('first_frame_ms'),'g_ms':g['avg_launch_ms'],'g_fb':g['fallback_avg_ms'],'c_ms':k['avg_launch_ms'],'c_fb':k['fallback_avg_ms'],'frac':d['roofline']['frac'],'sha':d.get('image_sha16')}))" >> $D/ab.jsonl
      tail -1 $D/ab.jsonl
    done
  done
done
