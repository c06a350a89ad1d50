#!/bin/bash
# BLAKE3 dual-issue test: clocks per VALU of the compression streams
# (kinds 100-106 of issue_rates.hip) at 1-8 waves per SIMD, then one PMC pass for the share
# of VALU instructions issued in pairs.  TAG=r05_x bash scripts/micro/dual_issue.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-dual}
K=${KINDS:-0,3,100,101,102,103,104,105,106}
timeout -k 10 180 scripts/micro/_bin/issue_rates $K > gpurun_out/${T}_issue_b3.json || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU -d gpurun_out/${T}_pmc_b3 -o run --output-format csv \
  -- scripts/micro/_bin/issue_rates ${PMC_KINDS:-100,102,104,106} > gpurun_out/${T}_pmc_b3.log 2>&1 || { tail -5 gpurun_out/${T}_pmc_b3.log; exit 1; }
python3 scripts/micro/dual_summary.py gpurun_out/${T}_pmc_b3 > gpurun_out/${T}_dual_b3.json
echo dual ok
