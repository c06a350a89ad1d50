# queue_probe over stream kinds x idle/busy fillers at 4 hardware queues (round 6)
cd $GRAFT_REPO_ROOT
for q in 4; do for k in 0 1 3; do for f in 3 8 16; do for b in 0 1; do
GPU_MAX_HW_QUEUES=$q timeout -k 5 30 scripts/micro/_bin/queue_probe $k 3 $f 40 $b | tail -1 | sed "s/^{/{\"hwq\": $q, /"
done; done; done; done
