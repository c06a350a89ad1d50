cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v33
for rep in 1 2; do
for cd in 10: 10:--profile-first 1: 1:--profile-first; do
    IFS=: read d pf <<< "$cd"
    f=gpurun_out/${T}_c2_d${d}${pf}_$rep
    timeout -k 10 240 python -u bench.py --config c2 --steps 20 --warmup 5 --depth $d $pf --no-cpu-baseline \
      --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || exit $?
    python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['stages_ms'], d['roofline']['scan_kernel']['cold_hbm']['ms'])" $f.json
done
done
