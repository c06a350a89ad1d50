cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r05_v7}
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_robust.py -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_stream.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_stream.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_stream.log
VARIANTS="prod b3pin" CONFIGS="c3" ROUNDS=3 STEPS=20 TESTS="tests/test_gpu_parity.py" TAG=${T}_b3 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 400 python3 -u scripts/stream_shape.py --hw-queues 4 --shapes 0:0 > gpurun_out/${T}_stream_rule_q4.json 2> gpurun_out/${T}_stream_rule_q4.err || { tail -20 gpurun_out/${T}_stream_rule_q4.err; exit 1; }
cat gpurun_out/${T}_stream_rule_q4.err
echo done
