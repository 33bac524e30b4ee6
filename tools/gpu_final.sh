set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-r6f2} TESTS=1 SMOKE=1 BENCH=1 PROF=1 CONFIGS="c3 c4 c5" bash tools/gpu_round.sh
