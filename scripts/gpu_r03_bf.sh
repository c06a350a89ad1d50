#!/bin/bash
# Round 3 session BF: SHA-256 split consumers: two-block main-loop body (one readiness probe,
# toggled ring offsets, no prefetch guard) -- SHA parity tests, then configs
# 2 / 5 / 4 product vs HEAD (base), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_robust.py tests/test_gpu_stream.py tests/test_gpu_cas.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py > gpurun_out/r03_bf_tests.log 2>&1 || { tail -30 gpurun_out/r03_bf_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r03_bf_tests.log)"
for r in 1 2 3; do
  for cfg in c2 c5 c4; do
    for v in prod base; do
      if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
      timeout -k 10 300 python3 bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r03_bf_${cfg}_${v}_$r.json 2> gpurun_out/r03_bf_${cfg}_${v}_$r.err || { tail -3 gpurun_out/r03_bf_${cfg}_${v}_$r.err; exit 1; }
      python3 -c "
import json; l=json.loads(open('gpurun_out/r03_bf_${cfg}_${v}_$r.json').read().strip().splitlines()[-1])
f=l.get('roofline',{}).get('latency_floor') or {}
print('$cfg', '$v', $r, l['value'], l['stages_ms']['digest_timed'], f.get('frac'))" | tee -a gpurun_out/r03_bf_ab.txt
    done
  done
done
echo "rc=0"
