# round 6 v45: the N > 1 bench path with the final pipeline, rehearsed on the one GPU:
# two gloo ranks (host-copy gather), and one nccl rank (--dist-force)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 2 --depth 40 --no-cpu-baseline --no-concurrent > gpurun_out/r06_v45_g2_gloo.json 2> gpurun_out/r06_v45_g2_gloo.err || { tail -20 gpurun_out/r06_v45_g2_gloo.err; exit 1; }
python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/r06_v45_g2_gloo.json') if l.startswith('{')][-1];print('gloo x2', d['value'], d['n_gpus'], d.get('gather_check'), d['pipeline']['group'], d['pipeline']['lanes'], d['pipeline']['depth'])"
timeout -k 10 500 python -u bench.py --dist-force --steps 20 --warmup 5 --no-cpu-baseline --no-concurrent > gpurun_out/r06_v45_dist.json 2> gpurun_out/r06_v45_dist.err || { tail -20 gpurun_out/r06_v45_dist.err; exit 1; }
python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/r06_v45_dist.json') if l.startswith('{')][-1];print('nccl x1', d['value'], 'steady', d['pipeline']['steady_window']['GiBps'], d.get('gather_check'))"
