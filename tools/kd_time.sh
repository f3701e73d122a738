set -o pipefail
mkdir -p gpurun_out/kd
for kd in gpu host; do
  GI_HOST_KD=$([ $kd = host ] && echo 1 || echo 0) timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/kd/c2_$kd.log 2>&1 || exit 1
  echo "C2 $kd $(grep '^{' gpurun_out/kd/c2_$kd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["photon_map_s"], d["value"])')"
  GI_HOST_KD=$([ $kd = host ] && echo 1 || echo 0) timeout -k 10 300 python3 bench.py --scene stilllife.scn --res 128 --aa 0 --global-photons 2000000 --caustic-photons 10000000 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/kd/c4_$kd.log 2>&1 || exit 1
  echo "C4 $kd $(grep '^{' gpurun_out/kd/c4_$kd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["photon_map_s"], d["config"]["global_stored"], d["config"]["caustic_stored"], d["value"])')"
done
