#!/bin/bash
# Round 4 session F: persistent-scan schedule A/B (queue read at mid / late, static
# grid-stride, unit sizes) against the one-shot kernel, plus the coalescer at 2 sets.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/scan_ab.py --configs c2,c4,c5 --reps 5 > gpurun_out/r04f_scan_ab.json 2> gpurun_out/r04f_scan_ab.err || { tail -5 gpurun_out/r04f_scan_ab.err; exit 1; }
for v in static8 static16 late8 late16 spu16 spu32; do
  CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so timeout -k 10 300 python -u scripts/scan_ab.py --configs c2,c4,c5 --reps 5 > gpurun_out/r04f_scan_ab_$v.json 2> gpurun_out/r04f_scan_ab_$v.err || { tail -5 gpurun_out/r04f_scan_ab_$v.err; exit 1; }
done
timeout -k 10 300 python bench.py --concurrent-only --concurrent-reps 6 > gpurun_out/r04f_conc_coal2.json 2> gpurun_out/r04f_conc_coal2.err || exit 1
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r04f_scan_ab*.json")):
    d=json.loads(open(f).read())
    print(f.split("/")[-1], {k:v["ms"] for k,v in d.items() if isinstance(v,dict)})
PY
cat gpurun_out/r04f_conc_coal2.json
echo "rc=0"
