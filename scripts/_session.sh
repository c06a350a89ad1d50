cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS="bench configs trace" TAG=r05_v9 bash scripts/gpu_validate.sh
