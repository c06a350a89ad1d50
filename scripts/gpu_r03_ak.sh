#!/bin/bash
# Round 3 session AK: SHA-256 LDS ring sized to the workgroup kinds launched (8 rows for
# quads only, 32 with pairs) -- SHA / stream / config tests, then config 2 single batch +
# batches in flight + host-to-host, and the stream bench, product (lean) vs 64 rows (fat).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_robust.py tests/test_gpu_stream.py tests/test_gpu_cas.py tests/test_gpu_configs.py > gpurun_out/r03_ak_tests.log 2>&1 || { tail -30 gpurun_out/r03_ak_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r03_ak_tests.log)"
for r in 1 2; do
  for v in prod fat; do
    if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
    timeout -k 10 300 python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r03_ak_${v}_$r.json 2> gpurun_out/r03_ak_${v}_$r.err || { tail -3 gpurun_out/r03_ak_${v}_$r.err; exit 1; }
    python3 -c "
import json; l=json.loads(open('gpurun_out/r03_ak_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', $r, l['value'], l['stages_ms']['digest_timed'], l.get('concurrent'), l.get('e2e'))" | tee -a gpurun_out/r03_ak_ab.txt
    timeout -k 10 300 python3 -u scripts/stream_bench.py > gpurun_out/r03_ak_stream_${v}_$r.json 2> gpurun_out/r03_ak_stream_${v}_$r.err || { tail -3 gpurun_out/r03_ak_stream_${v}_$r.err; exit 1; }
    echo "stream $v $r $(tail -1 gpurun_out/r03_ak_stream_${v}_$r.json)" | tee -a gpurun_out/r03_ak_ab.txt
  done
done
echo "rc=0"
