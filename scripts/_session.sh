cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS="tests slow smoke bench configs" TAG=r05_v18 bash scripts/gpu_validate.sh
