# r06t: the global list's row sort with 8 (in-tree: 30 key bits, no valid count), 10 and 11 radix
# bits per onesweep pass (exp/r10, exp/r11) against exp/base (31 bits, 8-bit passes): kernel-trace
# stats of one warm C2 frame each, then two interleaved rounds of C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06t
mkdir -p $D
: > $D/ab.jsonl
declare -A LIB=([base]=$GRAFT_REPO_ROOT/exp/base/libgi_amd.so [r8]= [r10]=$GRAFT_REPO_ROOT/exp/r10/libgi_amd.so [r11]=$GRAFT_REPO_ROOT/exp/r11/libgi_amd.so)
for v in base r8 r10 r11; do
  GI_AMD_LIB=${LIB[$v]} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/$v -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/$v.prof.log 2>&1 || { tail -20 $D/$v.prof.log; exit 1; }
  echo "$v prof done"
done
for r in 1 2; do
  for v in base r8 r10 r11; do
    GI_AMD_LIB=${LIB[$v]} timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/$v.$r.log 2>&1 || { tail -5 $D/$v.$r.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('$D/$v.$r.log').read().strip().splitlines()[-1])
g=d['roofline']['global']
print(json.dumps({'v':'$v','round':$r,'ms':d['ms_per_step'],'g_ms':g['avg_launch_ms'],'sha':d.get('image_sha16')}))" >> $D/ab.jsonl
    tail -1 $D/ab.jsonl
  done
done
