#!/bin/bash
# Round 3 session AD: lean split-consumer bookkeeping (CG_SHA_LEAN=1: no per-lane selects
# while every chunk runs, publish without exec masking) vs the product -- SHA parity tests
# on the variant, then config 2 alternating builds and config 5 once each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_lean.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sha or SHA or digest or batch or quad" > gpurun_out/r03_ad_tests.log 2>&1 || { tail -30 gpurun_out/r03_ad_tests.log; exit 1; }
echo "lean tests: $(tail -1 gpurun_out/r03_ad_tests.log)"
for r in 1 2 3; do
  for v in prod lean; do
    if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
    timeout -k 10 200 python3 bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/r03_ad_${v}_$r.json 2> gpurun_out/r03_ad_${v}_$r.err || { tail -3 gpurun_out/r03_ad_${v}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['stages_ms']['digest_timed'],d['roofline']['latency_floor']['frac'])" gpurun_out/r03_ad_${v}_$r.json $v
    cat gpurun_out/r03_ad_${v}_$r.json >> gpurun_out/r03_ad_all.jsonl
  done
done
for v in prod lean; do
  if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
  timeout -k 10 300 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/r03_ad_${v}_c5.json 2> gpurun_out/r03_ad_${v}_c5.err || { tail -3 gpurun_out/r03_ad_${v}_c5.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],'c5',d['value'],d['stages_ms']['digest_timed'])" gpurun_out/r03_ad_${v}_c5.json $v
  cat gpurun_out/r03_ad_${v}_c5.json >> gpurun_out/r03_ad_all.jsonl
done
echo "rc=0"
