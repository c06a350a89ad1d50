#!/bin/bash
# Round 3 session X: BLAKE3 group map fused into the walk + descriptor assembly (no k_b3_plan
# launch) -- the BLAKE3 parity tests, then config 3 alternating the fused build (product)
# with the unaligned-load variant (CG_B3_UNALIGNED=1 on top of it) and a k_b3_plan build
# (CG_B3_FUSED_PLAN=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -k "blake3 or B3 or b3 or config3 or group_map" > gpurun_out/r03_x_tests.log 2>&1 || { tail -30 gpurun_out/r03_x_tests.log; exit 1; }
echo "product tests: $(tail -1 gpurun_out/r03_x_tests.log)"
CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_b3u.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -k "blake3 or B3 or b3 or config3 or group_map" > gpurun_out/r03_x_tests_b3u.log 2>&1 || { tail -30 gpurun_out/r03_x_tests_b3u.log; exit 1; }
echo "b3u tests: $(tail -1 gpurun_out/r03_x_tests_b3u.log)"
for r in 1 2 3; do
  for v in prod b3u plan; do
    if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
    timeout -k 10 200 python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-concurrent > gpurun_out/r03_x_${v}_$r.json 2> gpurun_out/r03_x_${v}_$r.err || { echo "bench $v failed"; tail -3 gpurun_out/r03_x_${v}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['ms_per_step'],d['stages_ms'])" gpurun_out/r03_x_${v}_$r.json $v
    cat gpurun_out/r03_x_${v}_$r.json >> gpurun_out/r03_x_all.jsonl
  done
done
echo "rc=0"
