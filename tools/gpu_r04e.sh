# r04: persistent continuation kernel parity + A/B; C3 Monte Carlo kernel stats with the
# persistent kernels on / off; fp64 VALU utilisation of the path kernels (tools/pmc_fp64.py)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04e && mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -m gpu -x -v --timeout 300 --timeout-method thread -k "continuation_queue or full_gi or batch_rerun" > $D/tests.log 2>&1 || { tail -30 $D/tests.log; exit 1; }
tail -2 $D/tests.log
C3="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline"
for v in "1024 1024" "1024 0" "0 0"; do
  set -- $v
  GI_MC_PERSIST=$1 GI_CONT_PERSIST=$2 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $D/c2_$1_$2.log 2>&1 || { tail -5 $D/c2_$1_$2.log; exit 1; }
  echo "C2 mc=$1 cont=$2 $(tail -1 $D/c2_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["image_sha16"])')"
  GI_MC_PERSIST=$1 GI_CONT_PERSIST=$2 timeout -k 10 300 python3 -u bench.py $C3 --steps 2 --warmup 1 > $D/c3_$1_$2.log 2>&1 || { tail -5 $D/c3_$1_$2.log; exit 1; }
  echo "C3 mc=$1 cont=$2 $(tail -1 $D/c3_$1_$2.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["image_sha16"])')"
done
for v in "1024 1024" "0 0"; do
  set -- $v
  GI_MC_PERSIST=$1 GI_CONT_PERSIST=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c3prof_$1_$2 -o run -- python3 bench.py $C3 --steps 1 --warmup 1 > $D/c3prof_$1_$2.log 2>&1 || { tail -5 $D/c3prof_$1_$2.log; exit 1; }
done
TAG=_c3 BENCH_ARGS="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000" bash tools/gpu_pmc_fp64.sh
TAG=_c2 bash tools/gpu_pmc_fp64.sh
echo ok
