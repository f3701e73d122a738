# r06 cold first frame: ONE shard bench as the first GPU process on a fresh box (the GPU idle
# before it), so first_frame_ms is the drop-in CLI's one-frame cost without a previous process's
# memory being cleared under it. usage: bash tools/r06/gpu_cold.sh c4|c5 OUTDIR
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/$2
mkdir -p $D
case $1 in
  c4) A=(--steps 2 --warmup 1 --scene stilllife.scn --res 2048 --global-photons 2000000 --caustic-photons 10000000 --shard 0/8);;
  c5) A=(--steps 2 --warmup 1 --scene teapot.scn --res 4096 --aa 3 --global-photons 8000000 --caustic-photons 0 --extra "-dof 4 12.2282 0.025 -no_caustic" --shard 1/8);;
esac
rocm-smi --showmemuse > $D/$1_smi_before.txt 2>&1 || true
timeout -k 10 600 python3 -u bench.py "${A[@]}" --no-cpu-baseline > $D/$1_cold.log 2>&1 || { tail -5 $D/$1_cold.log; exit 1; }
tail -1 $D/$1_cold.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'cfg':'$1','first_frame_ms':d['first_frame_ms'],'step_ms':d['step_ms'],'ms_per_step':d['ms_per_step'],'photon_map_s':d['config']['photon_map_s']}))" | tee $D/$1_cold.json
