cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
VARIANTS="prod +--split-mode=1,--bound-cus=32 +--split-mode=1,--bound-cus=64 +--split-mode=1" CONFIGS="c4 c5" ROUNDS=2 STEPS=10 TESTS=none TAG=r05_v12 bash scripts/gpu_ab.sh || exit 1
