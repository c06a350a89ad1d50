cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r05_v3}
timeout -k 10 600 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_fast.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_fast.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_fast.log
TAG=${T}_dual bash scripts/micro/dual_issue.sh || exit 1
LIBS="prod spill" ROUNDS=3 CONFIGS=c2,c4,c5 KERNELS=0 TAG=${T}_scan bash scripts/scan_ab_libs.sh || exit 1
VARIANTS="prod +--bound-priority" CONFIGS="c4 c5 c2" ROUNDS=2 STEPS=10 TESTS=none TAG=$T bash scripts/gpu_ab.sh || exit 1
timeout -k 10 400 python3 -u scripts/stream_shape.py --hw-queues 4 > gpurun_out/${T}_stream_shape_q4.json 2> gpurun_out/${T}_stream_shape_q4.err || { tail -20 gpurun_out/${T}_stream_shape_q4.err; exit 1; }
cat gpurun_out/${T}_stream_shape_q4.err
echo done
