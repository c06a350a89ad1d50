#!/bin/bash
# Round 3 session AN: SHA-256 consumer loop-head waits: HEAD (base) vs block-0 wait before
# the loop (pre) vs that + the one-lane rounds pinned between the readiness probe and its
# check (pin, the product candidate); configs 4 / 2 / 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sha or SHA or workgroup or digest" > gpurun_out/r03_an_tests.log 2>&1 || { tail -30 gpurun_out/r03_an_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r03_an_tests.log)"
for cfg in c4 c2 c5 c4; do
  for v in base pre pin; do
    export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so
    timeout -k 10 300 python3 bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r03_an_${cfg}_${v}.json 2> gpurun_out/r03_an_${cfg}_${v}.err || { tail -3 gpurun_out/r03_an_${cfg}_${v}.err; exit 1; }
    python3 -c "
import json; l=json.loads(open('gpurun_out/r03_an_${cfg}_${v}.json').read().strip().splitlines()[-1])
f=l.get('roofline',{}).get('latency_floor') or {}
print('$cfg', '$v', l['value'], l['stages_ms']['digest_timed'], f.get('frac'))" | tee -a gpurun_out/r03_an_ab.txt
  done
done
echo "rc=0"
