cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v40
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_robust.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
VARIANTS="prod twostream" CONFIGS="c2 c5" ROUNDS=2 STEPS=20 TESTS=none TAG=$T bash scripts/gpu_ab.sh || exit 1
for v in prod twostream; do
  lib=""; [ $v = twostream ] && lib=chunker_amd/_ab/libchunker_amd_twostream.so
  CHUNKER_AMD_LIB=$lib timeout -k 10 400 python -u bench.py --concurrent-only --concurrent 12,16,32 --concurrent-reps 6 > gpurun_out/${T}_conc_$v.json 2> gpurun_out/${T}_conc_$v.err || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/${T}_conc_$v.json'))['concurrent']
for k in ('K12','K16','K32'):
    x=d[k+'_detail'];print('$v', k, 'merged', x['merged']['GiBps'], x['merged']['p99'], 'per_batch', x['per_batch']['GiBps'], x['per_batch']['p99'])"
done
