set -e
cd $GRAFT_REPO_ROOT
for q in 4 8; do for k in 0 1 2 3; do for f in 0 8; do
GPU_MAX_HW_QUEUES=$q timeout -k 5 30 scripts/micro/_bin/queue_probe $k 3 $f 40 | tail -1 | sed "s/^{/{\"hwq\": $q, /"
done; done; done > gpurun_out/r06_queue_probe.jsonl
cat gpurun_out/r06_queue_probe.jsonl
