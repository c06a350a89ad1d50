cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v52
out=gpurun_out/${T}_queues.txt
: > $out
for qd in 4:2 4:4 4:6 4:8 4:10 4:14 4:16 8:10 8:14 16:14 16:16; do
    IFS=: read q d <<< "$qd"
    f=gpurun_out/${T}_q${q}_d$d
    timeout -k 10 240 python -u bench.py --config c2 --steps 20 --warmup 5 --hw-queues $q --depth $d --no-cpu-baseline \
      --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 scripts/depth_row.py $f.json c2 "q$q d$d" | tee -a $out
done
