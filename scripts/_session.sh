cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
VARIANTS="prod +--chain-bound,--digest-cus=240 +--chain-bound,--digest-cus=224 +--digest-cus=240" CONFIGS="c4 c5 c2" ROUNDS=2 STEPS=20 TESTS=none TAG=r05_v17 bash scripts/gpu_ab.sh || exit 1
