# A/B of experiment builds (tools/exp_build.sh) on one workload: for each library in $LIBS
# (";"-separated, "default" = the in-tree build) one bench run; prints value, ms and image hash.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
IFS=';' read -ra LL <<< "${LIBS:-default}"
for l in "${LL[@]}"; do
  if [ "$l" = "default" ]; then unset GI_AMD_LIB; else export GI_AMD_LIB=$l; fi
  timeout -k 10 300 python3 bench.py ${BENCH_ARGS:-} --steps ${STEPS:-1} --warmup ${WARMUP:-1} --no-cpu-baseline > /tmp/ab.log 2>&1 || { tail -20 /tmp/ab.log; exit 1; }
  grep '^{' /tmp/ab.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l', d['value'], d['ms_per_step'], d['image_sha16'])"
done
