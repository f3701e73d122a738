# r06o: row_keys_kernel at 64 rows per wave, surface keys without indexed arrays: exactness
# (launch order tests), kernel-trace stats of one warm C2 frame with and without GI_SURF_KEY,
# then interleaved C2 / C3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r06o
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_render.py -k "launch_order or render" > $D/pytest.log 2>&1 || { tail -20 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/base -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/base.log 2>&1 || { tail -20 $D/base.log; exit 1; }
GI_SURF_KEY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/sk -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $D/sk.log 2>&1 || { tail -20 $D/sk.log; exit 1; }
OUT=r06o_ab ROUNDS=2 CFGS="c2 c3" VAR=GI_SURF_KEY=1 bash tools/r06/ab.sh
