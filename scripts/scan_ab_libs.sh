#!/bin/bash
# K1 A/B across compile-time variants: scripts/scan_ab.py once per library, in the order
# given, repeated ROUNDS times (alternating, one box):
#   LIBS="prod prio pf4" ROUNDS=2 TAG=r04_x bash scripts/scan_ab_libs.sh
# "prod" is the product library; other names are chunker_amd/_ab/libchunker_amd_NAME.so
# (scripts/build_variant.sh).  KERNELS: cg_test_scan_kernel values (default 0 = the
# product's choice per size).  Prints one line per (round, lib) with the median ms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-scan_ab}
for r in $(seq 1 "${ROUNDS:-2}"); do
  for v in ${LIBS:?set LIBS}; do
    lib=""; [ "$v" = prod ] || lib=chunker_amd/_ab/libchunker_amd_$v.so
    out=gpurun_out/${TAG}_${v}_$r.json
    CHUNKER_AMD_LIB=$lib timeout -k 10 300 python -u scripts/scan_ab.py --configs ${CONFIGS:-c2,c4,c5} --reps ${REPS:-5} --kernels ${KERNELS:-0} > $out 2> ${out%.json}.err || { tail -5 ${out%.json}.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$out').read()); print('$r $v', {k:v['ms'] for k,v in d.items() if isinstance(v,dict)})"
  done
done
echo "rc=0"
