# round 6 v44: final validation of the shipped build (BLAKE3 on three boundary streams, staggering off)
# fast + slow GPU suites, smoke, default bench lines c2-c5, kernel traces, config-2 PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
STEPS="tests slow smoke bench configs trace" TAG=r06_v44 bash scripts/gpu_validate.sh || exit $?
STEPS=20 CFG=c2 TAG=r06_v44_pmc_c2 bash scripts/gpu_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out r06_v44_pmc_c2 > gpurun_out/r06_v44_pmc_c2.json
