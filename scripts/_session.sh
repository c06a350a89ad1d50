cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v37
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "stream or push" > gpurun_out/${T}_stream_tests.log 2>&1 || { tail -20 gpurun_out/${T}_stream_tests.log; exit 1; }
tail -1 gpurun_out/${T}_stream_tests.log
for q in 4 16; do
  timeout -k 10 300 python -u scripts/stream_shape.py --hw-queues $q --shapes 0:0 > gpurun_out/${T}_stream_q$q.json 2> gpurun_out/${T}_stream_q$q.err || exit 1
  cut -c1-400 gpurun_out/${T}_stream_q$q.json
done
