#!/bin/bash
# Round 3 session T: batch parts (BLAKE3 scan/digest overlap) -- parity tests for the parts
# (historical: the --parts option and the batch-parts path it measured were reverted after this session)
# path, then config 3 at parts = 1 / 2 / 4 / 8 and the default, a kernel trace of the default, and
# the RCCL gather path rehearsed at one rank (bench.py --dist-force).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parts.py > gpurun_out/r03_t_parts_tests.log 2>&1 \
 && echo "parts tests ok" \
 && for k in 1 2 4 8 0; do timeout -k 10 200 python3 bench.py --config c3 --no-concurrent --no-cpu-baseline --parts $k > gpurun_out/r03_t_c3_p$k.json 2> gpurun_out/r03_t_c3_p$k.err || exit 1; python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'],d['batch_parts'],d['stages_ms'])" gpurun_out/r03_t_c3_p$k.json $k; done \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03_t_c3" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 5 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/prof_r03_t_c3.log 2>&1 \
 && echo "rocprof ok" \
 && timeout -k 10 300 python3 bench.py --gpus 1 --dist-force --dist-backend nccl --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/r03_t_nccl1.json 2> gpurun_out/r03_t_nccl1.err \
 && cat gpurun_out/r03_t_nccl1.json
rc=$?; tail -5 gpurun_out/r03_t_parts_tests.log; echo "rc=$rc"; exit $rc
