#!/bin/bash
# Round 3 session AY: SHA-256 LDS ring sized to the kinds launched (lean), re-run with the
# round code aligned (v32's A/B moved the asm stream by 4 bytes): SHA tests on lean, then
# config 2 single batch + 8 / 32 in flight, product vs lean, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_lean.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stream.py -k "sha or SHA or workgroup or digest or config or stream" > gpurun_out/r03_ay_tests.log 2>&1 || { tail -30 gpurun_out/r03_ay_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r03_ay_tests.log)"
for r in 1 2; do
  for v in prod lean; do
    if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
    timeout -k 10 300 python3 bench.py --config c2 --steps 8 --warmup 2 --no-cpu-baseline --e2e '' > gpurun_out/r03_ay_${v}_$r.json 2> gpurun_out/r03_ay_${v}_$r.err || { tail -3 gpurun_out/r03_ay_${v}_$r.err; exit 1; }
    python3 -c "
import json; l=json.loads(open('gpurun_out/r03_ay_${v}_$r.json').read().strip().splitlines()[-1])
c=l.get('concurrent') or {}
print('c2', '$v', $r, l['value'], l['stages_ms']['digest_timed'], c.get('K8'), c.get('K32'))" | tee -a gpurun_out/r03_ay_ab.txt
  done
done
echo "rc=0"
