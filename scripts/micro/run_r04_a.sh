#!/bin/bash
# Round 4 session A: VALU issue rates per SIMD (scripts/micro/issue_rates.hip) and the
# box's rocprofv3 counter list.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 scripts/micro/_bin/issue_rates > gpurun_out/r04_issue_rates.json 2> gpurun_out/r04_issue_rates.err \
  && echo "issue ok" \
  && timeout -k 10 120 rocprofv3 -L > gpurun_out/r04_counters.txt 2>&1; rc=$?
tail -c 3000 gpurun_out/r04_issue_rates.json
echo "rc=$rc"
exit $rc
