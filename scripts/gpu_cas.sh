#!/bin/bash
# CAS / Node::put session: CAS parity tests first, then the whole GPU suite, then the
# Node::put bench (c2, c4) and a rocprofv3 kernel trace of the c2 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 300 python -u -m pytest tests/test_gpu_cas.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_cas.log 2>&1 \
 && echo "cas tests ok" \
 && timeout -k 10 600 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 \
 && echo "gpu tests ok" \
 && timeout -k 10 240 python scripts/cas_bench.py --config c2 > gpurun_out/cas_c2.json 2> gpurun_out/cas_c2.err && cat gpurun_out/cas_c2.json \
 && timeout -k 10 300 python scripts/cas_bench.py --config c4 --steps 2 --cpu-sample-nars 0 > gpurun_out/cas_c4.json 2> gpurun_out/cas_c4.err && cat gpurun_out/cas_c4.json \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${TAG}_cas_c2" -o run --output-format csv -- python3 "$R/scripts/cas_bench.py" --config c2 --steps 2 --cpu-sample-nars 0 > gpurun_out/prof_${TAG}_cas_c2.log 2>&1 \
 && echo "rocprof ok"
rc=$?
echo "rc=$rc"
tail -5 gpurun_out/pytest_cas.log
tail -3 gpurun_out/pytest_gpu.log
exit $rc
