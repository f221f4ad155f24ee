set -o pipefail
# Multi-rank bench rehearsal on ONE MI355X: ranks share the card, control plane over gloo (GA_DIST_BACKEND); checks the slab pipeline end to end, not scaling.
cd /root/repo
mkdir -p gpurun_out/dist
export GA_DIST_BACKEND=gloo
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --workload c2 --steps 3 --warmup 1 > gpurun_out/dist/c2x2.json 2> gpurun_out/dist/c2x2.err || { tail -20 gpurun_out/dist/c2x2.err; exit 1; }
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 3 --workload c5 --steps 3 --warmup 1 > gpurun_out/dist/c5x3.json 2> gpurun_out/dist/c5x3.err || { tail -20 gpurun_out/dist/c5x3.err; exit 1; }
# score-only slabs (the lane-skewed kernel), 2 and 4 ranks
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --workload c4r --steps 3 --warmup 1 > gpurun_out/dist/c4rx2.json 2> gpurun_out/dist/c4rx2.err || { tail -20 gpurun_out/dist/c4rx2.err; exit 1; }
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --workload c4r --steps 3 --warmup 1 > gpurun_out/dist/c4rx4.json 2> gpurun_out/dist/c4rx4.err || { tail -20 gpurun_out/dist/c4rx4.err; exit 1; }
timeout -k 10 240 python bench.py --workload c4r --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dist/c4rx1.json 2> gpurun_out/dist/c4rx1.err || { tail -20 gpurun_out/dist/c4rx1.err; exit 1; }
for f in c2x2 c5x3 c4rx1 c4rx2 c4rx4; do tail -c 700 gpurun_out/dist/$f.json; echo; done
