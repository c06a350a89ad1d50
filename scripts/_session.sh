cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_robust.py -m gpu > gpurun_out/r05_v49_robust.log 2>&1 || { tail -30 gpurun_out/r05_v49_robust.log; exit 1; }
tail -1 gpurun_out/r05_v49_robust.log
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_robust.py -m gpu -k "lone or spin_guard_reaches" > gpurun_out/r05_v49_robust_q16.log 2>&1 || { tail -30 gpurun_out/r05_v49_robust_q16.log; exit 1; }
tail -1 gpurun_out/r05_v49_robust_q16.log
