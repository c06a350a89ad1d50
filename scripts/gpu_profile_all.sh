#!/bin/bash
# One GPU session: tests + default bench + rocprofv3 kernel-trace summary (gpu_check.sh),
# then PMC passes for configs c2 and c3 (gpu_pmc.sh).  Stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r01} bash scripts/gpu_check.sh \
 && CFG=c2 TAG=pmc_c2 bash scripts/gpu_pmc.sh \
 && CFG=c3 TAG=pmc_c3 bash scripts/gpu_pmc.sh \
 && python3 scripts/pmc_summary.py gpurun_out pmc_c2 > gpurun_out/pmc_c2.json \
 && python3 scripts/pmc_summary.py gpurun_out pmc_c3 > gpurun_out/pmc_c3.json \
 && echo "profile-all ok"
