cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v60
out=gpurun_out/${T}_var.txt
: > $out
for rep in 1 2 3; do
for d in 20 16 12; do
    f=gpurun_out/${T}_d${d}_$rep
    timeout -k 10 240 python -u bench.py --config c2 --steps 20 --warmup 5 --depth $d --no-cpu-baseline \
      --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 scripts/depth_row.py $f.json c2 "q22 d$d r$rep" | tee -a $out
done
done
