# round 6 v33: PMC passes of the product's merged digest launches (c2: 20 batches per launch;
# c4 / c5: 2), no stage profile, so the per-launch traffic matches the bench line's launch
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in c2 c4 c5; do
  if [ $c = c2 ]; then st=20; else st=2; fi
  STEPS=$st CFG=$c TAG=r06_v33_pmc_$c bash scripts/gpu_pmc.sh || exit $?
  python3 scripts/pmc_summary.py gpurun_out r06_v33_pmc_$c > gpurun_out/r06_v33_pmc_$c.json
  python3 -c "
import json
d=json.load(open('gpurun_out/r06_v33_pmc_$c.json'))
for k,v in d.items():
    if 'sha256' in k or 'scan_flat' in k: print('$c', k, v.get('fetch_bytes_x2'), v.get('write_bytes'), v.get('SQ_WAVES'), v.get('SQ_INSTS_VALU'))"
done
