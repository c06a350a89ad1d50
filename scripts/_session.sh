cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r05_v3}
timeout -k 10 600 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_fast.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_fast.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_fast.log
TAG=${T}_dual bash scripts/micro/dual_issue.sh || exit 1
VARIANTS="prod +--split-mode=2 +--bound-priority +--no-overlap" CONFIGS="c2 c3 c4 c5" ROUNDS=1 STEPS=10 TESTS=none TAG=$T bash scripts/gpu_ab.sh || exit 1
echo done
