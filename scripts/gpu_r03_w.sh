#!/bin/bash
# Round 3 session W: BLAKE3 leaf blocks loaded with unaligned dwordx4 (no v_alignbyte
# realignment, CG_B3_UNALIGNED=1) vs the product -- BLAKE3 parity tests on the variant,
# then config 3 alternating builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_b3u.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -k "blake3 or B3 or b3 or config3" > gpurun_out/r03_w_tests.log 2>&1 || { tail -20 gpurun_out/r03_w_tests.log; exit 1; }
echo "variant tests: $(tail -1 gpurun_out/r03_w_tests.log)"
for r in 1 2 3; do
  for v in prod b3u; do
    if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
    timeout -k 10 200 python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-concurrent > gpurun_out/r03_w_${v}_$r.json 2> gpurun_out/r03_w_${v}_$r.err || { echo "bench $v failed"; tail -3 gpurun_out/r03_w_${v}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['stages_ms'])" gpurun_out/r03_w_${v}_$r.json $v
    cat gpurun_out/r03_w_${v}_$r.json >> gpurun_out/r03_w_all.jsonl
  done
done
echo "rc=0"
