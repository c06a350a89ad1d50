cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v26
out=gpurun_out/${T}_tiers_fill_ab.txt
: > $out
for rep in 1 2; do
for cd in c4:4:850,600,950,700 c4:4:850,600,980,750 c4:4:850,600,1000,800 c4:4:850,600,1000,1000 c4:4:850,600,980,600 c4:4:850,600,0,0 c4:2:850,600,950,700 c4:8:850,600,950,700; do
    IFS=: read cfg d t <<< "$cd"
    f=gpurun_out/${T}_${cfg}_d${d}_t${t//,/_}_$rep
    timeout -k 10 240 python -u bench.py --config $cfg --steps 20 --warmup 5 --depth $d --sha-tiers $t --no-cpu-baseline \
      --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || exit $?
    python3 scripts/depth_row.py $f.json $cfg "$d t$t" | tee -a $out
done
done
