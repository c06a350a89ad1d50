#!/bin/bash
# PMC counter passes (scripts/gpu_pmc.sh: one rocprofv3 --pmc pass per counter group, no
# trace domains) for every bench config, summarised per kernel (scripts/pmc_summary.py)
# into gpurun_out/${TAG}_pmc_<config>.json -- the files bench.py's `traffic` reads once
# copied under profiles/.  Stops at the first pass that dies.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${TAG:-r04}
for c in ${CONFIGS:-c2 c3 c4 c5}; do
  CFG=$c TAG=${TAG}_pmc_$c bash scripts/gpu_pmc.sh || exit $?
  python3 scripts/pmc_summary.py gpurun_out ${TAG}_pmc_$c > gpurun_out/${TAG}_pmc_$c.json || exit 1
  echo "pmc $c ok"
done
