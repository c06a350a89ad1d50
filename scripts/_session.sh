cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v11
CONFIGS="c4" TAG=${T}_prod bash scripts/gpu_pmc_all.sh || exit 1
CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_inplace.so CONFIGS="c2 c4" TAG=${T}_inplace bash scripts/gpu_pmc_all.sh || exit 1
echo done
