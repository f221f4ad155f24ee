set -o pipefail
# round 6: (1) the readlane micro v2 (lane selects >= 64); (2) the host tie-break table, sequential and
# threaded, on the box's cores; (3) C3-shape lane stamps with the lag probed at rows 256 / 1024 / 4096 / 16384
export TMPDIR=/tmp
O=gpurun_out/r6_probe2
mkdir -p $O
timeout -k 10 60 ./tools/micro/readlane_idx2 > $O/micro_readlane_idx2.txt 2>&1 || { cat $O/micro_readlane_idx2.txt; exit 1; }
cat $O/micro_readlane_idx2.txt
timeout -k 10 120 ./globalign_amd/_lib/ga_host_selftest bench 200001 > $O/rng_bench.txt 2>&1 || { cat $O/rng_bench.txt; exit 1; }
cat $O/rng_bench.txt
nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_c3td4.json 2> $O/stamps_c3td4.err || { tail -5 $O/stamps_c3td4.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/stamps_c3td4.json').read().strip().splitlines()[-1])
print('plain', round(d['fill_ms_plain'],3), 'dbg', round(d['fill_ms_dbg'],3))
for k,v in d['lag_by_row'].items(): print('lag at row', k, {a: round(b,2) for a,b in v.items()})
print(d['probe_m2'])
"
