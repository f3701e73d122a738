# r06k: C5 cold first frame with doubling buffer growth (fresh box, first process), then C2 / C4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06k
GI_LOG=1 timeout -k 10 600 python3 -u bench.py --steps 2 --warmup 1 --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 0 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8 --no-cpu-baseline > gpurun_out/r06k/c5.log 2>&1 || { tail -5 gpurun_out/r06k/c5.log; exit 1; }
tail -1 gpurun_out/r06k/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['first_frame_ms'], d['step_ms'])"
GI_LOG=1 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06k/c2.log 2>&1 || { tail -5 gpurun_out/r06k/c2.log; exit 1; }
tail -1 gpurun_out/r06k/c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['first_frame_ms'], d['step_ms'], d['image_sha16'])"
GI_LOG=1 timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --shard 0/8 --no-cpu-baseline > gpurun_out/r06k/c4.log 2>&1 || { tail -5 gpurun_out/r06k/c4.log; exit 1; }
tail -1 gpurun_out/r06k/c4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['first_frame_ms'], d['step_ms'])"
