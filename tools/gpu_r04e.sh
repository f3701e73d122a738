# r04: C3 Monte Carlo kernels: kernel stats with the persistent kernel on / off, its grid size,
# and the fp64 VALU utilisation of the path kernels (tools/pmc_fp64.py)
set -o pipefail
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && D=gpurun_out/r04e && mkdir -p $D
C3="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline"
for p in 1024 0; do
  GI_MC_PERSIST=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/c3_p$p -o run -- python3 bench.py $C3 --steps 1 --warmup 1 > $D/c3_p$p.log 2>&1 || { tail -5 $D/c3_p$p.log; exit 1; }
  echo "C3 persist=$p: $(grep -E 'mc_(persist_)?kernel' $D/c3_p$p/run_kernel_stats.csv | awk -F, '{s+=$3} END {print s/1e6 " ms mc"}')"
done
for p in 512 2048 4096; do
  GI_MC_PERSIST=$p timeout -k 10 300 python3 -u bench.py $C3 --steps 2 --warmup 1 > $D/c3_sweep_$p.log 2>&1 || { tail -5 $D/c3_sweep_$p.log; exit 1; }
  echo "C3 persist=$p $(tail -1 $D/c3_sweep_$p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["image_sha16"])')"
done
TAG=_c3 BENCH_ARGS="--scene jensen.scn --global-photons 2176 --caustic-photons 4000000" bash tools/gpu_pmc_fp64.sh
TAG=_c2 bash tools/gpu_pmc_fp64.sh
echo ok
