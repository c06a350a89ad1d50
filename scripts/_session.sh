cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
KINDS=100,125,127 PMC_KINDS=100,125,127 TAG=r05_v14_dual bash scripts/micro/dual_issue.sh || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/r05_v14_dual_issue_b3.json'))
for r in d['rows']: print(r['kind'], {k:v['cyc'] for k,v in r.items() if k.startswith('w')})
d=json.load(open('gpurun_out/r05_v14_dual_dual_b3.json'))
for r in d['rows']: print(r['kernel'][:20], r['w'], r['dual_frac'])
"
VARIANTS="prod b3asm" CONFIGS="c3" ROUNDS=3 STEPS=20 TESTS="tests/test_gpu_parity.py" TAG=r05_v14_b3 bash scripts/gpu_ab.sh || exit 1
