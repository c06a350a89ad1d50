#!/bin/bash
# Round 3 session U: SHA-256 LDS ring depth A/B (PC_RING 4 = product, 3, 2: 68 / 52 / 35 KB
# per workgroup -> 2 / 3 / 4 workgroups per CU in GPU-filling batches).  Per variant: the
# SHA parity tests, then configs 2, 4, 5 and config-2 batches in flight.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in prod r3 r2; do
  if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
  timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sha or digest or batch" > gpurun_out/r03_u_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -5 gpurun_out/r03_u_tests_$v.log; exit 1; }
  echo "tests $v ok: $(tail -1 gpurun_out/r03_u_tests_$v.log)"
  for c in c2 c4 c5; do
    timeout -k 10 200 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/r03_u_${v}_$c.json 2> gpurun_out/r03_u_${v}_$c.err || { echo "bench $v $c failed"; tail -3 gpurun_out/r03_u_${v}_$c.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],sys.argv[3],d['value'],d['stages_ms']['digest_timed'],d['roofline'].get('latency_floor',{}).get('workgroups'))" gpurun_out/r03_u_${v}_$c.json $v $c
  done
  timeout -k 10 300 python3 bench.py --config c2 --concurrent-only --concurrent 8,32 > gpurun_out/r03_u_${v}_conc.json 2> gpurun_out/r03_u_${v}_conc.err || { echo "conc $v failed"; exit 1; }
  echo "$v $(cat gpurun_out/r03_u_${v}_conc.json)"
done
echo "rc=0"
