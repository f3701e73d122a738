# r06r: caustic surface keys with 18-bit in-plane cells (in-tree) against 16-bit (exp/base), C4 / C3 / C2
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=r06r ROUNDS=1 CFGS="c4 c3 c2" bash tools/r06/ab.sh
