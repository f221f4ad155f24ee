# round 2: the walker's own accounting (tile waits, loads) inside the pipelined C3 steps, and alone
set -o pipefail
mkdir -p gpurun_out/exp
rm -f gpurun_out/exp/trace_c3_wdiag.jsonl
GA_PIPE_TRACE=gpurun_out/exp/trace_c3_wdiag.jsonl timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/wdiag.json 2> gpurun_out/exp/wdiag.err || { tail -20 gpurun_out/exp/wdiag.err; exit 1; }
python -c "
import json
rows=[json.loads(l) for l in open('gpurun_out/exp/trace_c3_wdiag.jsonl')][-10:]
for r in rows: print(r['k'], round(r['walk1']-r['walk0'],2), r['walker_us'], r['tile_wait_us'], r['tile_loads'], r['load_us_per_tile'])
"
timeout -k 10 120 python -u tools/walk_diag.py c3 > gpurun_out/exp/walk_diag_c3.json 2> gpurun_out/exp/walk_diag_c3.err || { tail -20 gpurun_out/exp/walk_diag_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/exp/walk_diag_c3.json'));r=d['runs'][-1];print('alone', {k:r[k] for k in ['walk_ms','tile_wait_us','load_us_per_tile','walker_clk_per_step','loads']})"
