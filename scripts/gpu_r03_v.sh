#!/bin/bash
# Round 3 session V: deeper SHA-256 rings for the latency-bound config 2 (PC_RING 6 / 8 vs 4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in prod r6 r8 prod; do
  if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
  timeout -k 10 200 python3 bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline --no-concurrent > gpurun_out/r03_v_${v}_c2.json 2> gpurun_out/r03_v_${v}_c2.err || { echo "bench $v failed"; tail -3 gpurun_out/r03_v_${v}_c2.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],d['value'],d['stages_ms']['digest_timed'],d['roofline']['latency_floor']['frac'])" gpurun_out/r03_v_${v}_c2.json $v
  cat gpurun_out/r03_v_${v}_c2.json >> gpurun_out/r03_v_all.jsonl
done
echo "rc=0"
