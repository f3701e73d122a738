# r04: block-chunked persistence for the Monte Carlo paths (GI_MC_CHUNK paths per thread from the
# block's own range): C2, C3, C4 shard 0/8 against the plain and global-counter kernels
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04m && timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04m/render_tests.log 2>&1 || { tail -30 gpurun_out/r04m/render_tests.log; exit 1; }
tail -1 gpurun_out/r04m/render_tests.log
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04m && mkdir -p $D
C3=(--scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline)
C4=(--scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --no-cpu-baseline --shard 0/8)
for v in "0 0" "4 0" "16 0" "64 0" "0 1024"; do
  set -- $v
  E="GI_MC_CHUNK=$1 GI_MC_PERSIST=$2"
  env GI_MC_CHUNK=$1 GI_MC_PERSIST=$2 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$1_$2.log 2>&1 || { tail -5 $D/c2_$1_$2.log; exit 1; }
  env GI_MC_CHUNK=$1 GI_MC_PERSIST=$2 timeout -k 10 300 python3 -u bench.py "${C3[@]}" --steps 2 --warmup 1 > $D/c3_$1_$2.log 2>&1 || { tail -5 $D/c3_$1_$2.log; exit 1; }
  env GI_MC_CHUNK=$1 GI_MC_PERSIST=$2 timeout -k 10 300 python3 -u bench.py "${C4[@]}" --steps 1 --warmup 1 > $D/c4_$1_$2.log 2>&1 || { tail -5 $D/c4_$1_$2.log; exit 1; }
  for c in c2 c3 c4; do echo "$c $E $(tail -1 $D/${c}_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["image_sha16"])')"; done
done
echo ok
