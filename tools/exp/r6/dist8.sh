set -o pipefail
# round 6: the bench's multi-rank path at 8 ranks sharing the one MI355X (gloo control), the
# c4r shape (1M x 16k, score only) in both edge modes against the oracle's cost, the edge preflight in each line;
# 1, 2, 4 ranks beside it.  Ranks sharing one card say nothing about scaling.
export GA_DIST_BACKEND=gloo
O=gpurun_out/r6_dist
mkdir -p $O
run() {
  n=$1; edge=$2; port=$3
  GA_SLAB_EDGE=$edge timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --workload c4r --steps 3 --warmup 1 > $O/c4rx${n}_$edge.json 2> $O/c4rx${n}_$edge.err || { tail -20 $O/c4rx${n}_$edge.err; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('$O/c4rx${n}_$edge.json') if l.startswith('{')][-1]
c=d['config']; e=c['edge_links']
print('c4r x$n $edge', round(d['ms_per_step'],2), 'ms', 'cost_ok', c['cost_matches_oracle'], 'ipc', e['ipc_agreed'], [b['transport'].split()[0] for b in e['boundaries']], e['ipc_errors'])
"
}
timeout -k 10 200 python bench.py --workload c4r --steps 3 --warmup 1 --no-cpu-baseline > $O/c4rx1.json 2> $O/c4rx1.err || { tail -20 $O/c4rx1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c4rx1.json').read().strip().splitlines()[-1]); print('c4r x1', round(d['ms_per_step'],2), 'ms', d['config']['cost_matches_oracle'])"
run 2 ipc 29611
run 4 ipc 29612
run 8 ipc 29613
run 8 bands 29614
