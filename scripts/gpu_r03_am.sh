#!/bin/bash
# Round 3 session AM: config 2 digest, HEAD (base) vs block-0 wait before the consumer loop
# only (pre) vs that + inline-asm readiness probe (probe).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for v in base pre probe; do
    export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so
    timeout -k 10 300 python3 bench.py --config c2 --steps 8 --warmup 2 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r03_am_${v}_$r.json 2> gpurun_out/r03_am_${v}_$r.err || { tail -3 gpurun_out/r03_am_${v}_$r.err; exit 1; }
    python3 -c "
import json; l=json.loads(open('gpurun_out/r03_am_${v}_$r.json').read().strip().splitlines()[-1])
f=l.get('roofline',{}).get('latency_floor') or {}
print('c2', '$v', $r, l['value'], l['stages_ms']['digest_timed'], f.get('frac'))" | tee -a gpurun_out/r03_am_ab.txt
  done
done
echo "rc=0"
