# round 2: 12 / 13 / 14 walk loader waves (GA_WALK_LOADERS): parity, the walker's accounting alone and in
# the pipeline
set -o pipefail
mkdir -p gpurun_out/exp
GA_WALK_LOADERS=14 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_many.py -x -q --timeout 240 --timeout-method thread > gpurun_out/exp/ldr.log 2>&1 || { tail -30 gpurun_out/exp/ldr.log; exit 1; }
tail -1 gpurun_out/exp/ldr.log
for L in 12 13 14; do
  rm -f gpurun_out/exp/trace_c3_ldr$L.jsonl
  GA_WALK_LOADERS=$L GA_PIPE_TRACE=gpurun_out/exp/trace_c3_ldr$L.jsonl timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --no-extra > gpurun_out/exp/ldr$L.json 2> gpurun_out/exp/ldr$L.err || { tail -20 gpurun_out/exp/ldr$L.err; exit 1; }
  python -c "
import json
d=json.load(open('gpurun_out/exp/ldr$L.json'))
rows=[json.loads(l) for l in open('gpurun_out/exp/trace_c3_ldr$L.jsonl')][-10:]
print('ldr$L c3', round(d['ms_per_step'],3), 'walk', round(d['walk_ms'],2), d['config']['traceback_pin']['matches_oracle'], 'tile_wait_us', round(sum(r['tile_wait_us'] for r in rows)/10,1))"
  GA_WALK_LOADERS=$L timeout -k 10 120 python -u tools/walk_diag.py c3 > gpurun_out/exp/wdl$L.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp/wdl$L.json'));r=d['runs'][-1];print('  alone', {k:r[k] for k in ['walk_ms','tile_wait_us','load_us_per_tile','loads']})"
  GA_WALK_LOADERS=$L timeout -k 10 120 python -u tools/walk_diag.py c5 > gpurun_out/exp/wdl5$L.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp/wdl5$L.json'));r=d['runs'][-1];print('  c5 alone', {k:r[k] for k in ['walk_ms','tile_wait_us','load_us_per_tile','loads']})"
done
