# Scratch GPU session (run as: gpurun -- bash scripts/_session.sh); the validation used at round end:
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS="tests slow smoke bench configs trace" TAG=r05_final bash scripts/gpu_validate.sh
