cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS="tests slow smoke bench configs trace" TAG=r05_v41 bash scripts/gpu_validate.sh
