cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
for c in c2 c4 c5; do
  CFG=$c TAG=r05_v35_pmc_$c bash scripts/gpu_pmc.sh || exit 1
  python3 scripts/pmc_summary.py gpurun_out r05_v35_pmc_$c > gpurun_out/r05_v35_pmc_$c.json || exit 1
done
