# r06 round-end, part B: C3 / C4 shard 0/8 / C5 shard 1/8 bench lines (final tree), then the
# global chunk k-NN's VALU instructions per wave on C2 (SQ counters; tools/pmc_fp64.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/final_b
mkdir -p $D
timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --scene jensen.scn --global-photons 2176 --caustic-photons 4000000 --no-cpu-baseline > $D/c3.log 2>&1 || { tail -5 $D/c3.log; exit 1; }
tail -1 $D/c3.log | cut -c1-200
timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --shard 0/8 --no-cpu-baseline > $D/c4.log 2>&1 || { tail -5 $D/c4.log; exit 1; }
tail -1 $D/c4.log | cut -c1-200
timeout -k 10 500 python3 -u bench.py --steps 2 --warmup 1 --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 0 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8 --no-cpu-baseline > $D/c5.log 2>&1 || { tail -5 $D/c5.log; exit 1; }
tail -1 $D/c5.log | cut -c1-200
TAG=_final bash tools/gpu_pmc_fp64.sh
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multi.py > $D/multi.log 2>&1 || { tail -20 $D/multi.log; exit 1; }
tail -1 $D/multi.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
