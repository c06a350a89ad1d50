# round 6 v21: final validation of the round's product (BLAKE3 leaves with the held tail line):
# fast + slow GPU suites, smoke, default bench lines c2-c5, kernel traces, config-3 PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
STEPS="tests slow smoke bench configs trace" TAG=r06_v21 bash scripts/gpu_validate.sh || exit $?
CFG=c3 TAG=r06_v21_pmc_c3 bash scripts/gpu_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out r06_v21_pmc_c3 > gpurun_out/r06_v21_pmc_c3.json
