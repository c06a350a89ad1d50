set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -k "diag_scan_variants" --timeout 120 --timeout-method thread > gpurun_out/pytest_variants.log 2>&1 && echo "variants ok" \
 && timeout -k 10 400 python -u scripts/diag_scan.py --variants "" --mode-variant 5 --modes 13,20,21,22,13,20 --spw 0 --configs c2,c5one,c4 --no-pattern --hash 1 > gpurun_out/diag_scan_split_sha.json 2>&1 && timeout -k 10 300 python -u scripts/diag_scan.py --variants "" --mode-variant 5 --modes 13,20 --spw 0 --configs c2 --no-pattern --hash 0 > gpurun_out/diag_scan_split.json 2> gpurun_out/diag_scan_split.err; rc=$?; cat gpurun_out/diag_scan_split_sha.json gpurun_out/diag_scan_split.json; tail -3 gpurun_out/pytest_variants.log; exit $rc
