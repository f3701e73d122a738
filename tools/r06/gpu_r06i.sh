# r06i: stream priorities (GI_SIDE_PRIO=1: the Monte Carlo side stream most urgent; -1: the main
# stream) against the default, C2 and C3
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=r06i_side ROUNDS=2 CFGS="c2 c3" VAR=GI_SIDE_PRIO=1 bash tools/r06/ab.sh || exit 1
OUT=r06i_main ROUNDS=1 CFGS="c2 c3" VAR=GI_SIDE_PRIO=-1 bash tools/r06/ab.sh
bash tools/gpu_pmc_icache.sh
