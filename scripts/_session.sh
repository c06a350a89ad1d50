cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v38
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "pipeline" > gpurun_out/${T}_pipeline.log 2>&1 || { tail -30 gpurun_out/${T}_pipeline.log; exit 1; }
tail -1 gpurun_out/${T}_pipeline.log
