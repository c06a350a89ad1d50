#!/bin/bash
# Round 3 session AJ: config 2 with the SHA-256 workgroups isolated one per CU (LDS pad on
# every launch, CG_SHA_PAD_ALWAYS) against the product (pad only when nwg <= 256).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in prod padall; do
    if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
    timeout -k 10 200 python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r03_aj_${v}_$r.json 2> gpurun_out/r03_aj_${v}_$r.err || { tail -3 gpurun_out/r03_aj_${v}_$r.err; exit 1; }
    python3 -c "
import json; l=json.loads(open('gpurun_out/r03_aj_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', $r, l['value'], l['ms_per_step'], l['stages_ms'], l.get('roofline',{}).get('latency_floor'))" | tee -a gpurun_out/r03_aj_ab.txt
  done
done
echo "rc=0"
