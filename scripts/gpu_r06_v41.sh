# round 6 v41: the shipped defaults (staggering off): fast GPU suite, smoke, default c2 line
set -o pipefail
cd $GRAFT_REPO_ROOT
STEPS="tests smoke bench" TAG=r06_v41 bash scripts/gpu_validate.sh || exit $?
