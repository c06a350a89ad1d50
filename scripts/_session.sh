cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS="tests slow smoke bench" TAG=r05_v15 bash scripts/gpu_validate.sh
