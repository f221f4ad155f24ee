# round 2: two-byte-word tile decode with one flags lookup: GPU suite, C5 walk diagnostics, C5 bench
set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/exp/cb2_suite.log 2>&1 || { tail -30 gpurun_out/exp/cb2_suite.log; exit 1; }
tail -1 gpurun_out/exp/cb2_suite.log
timeout -k 10 120 python -u tools/walk_diag.py c5 > gpurun_out/exp/walk_diag_c5.json 2> gpurun_out/exp/walk_diag_c5.err || { tail -20 gpurun_out/exp/walk_diag_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/exp/walk_diag_c5.json'));r=d['runs'][-1];print({k:r[k] for k in ['walk_ms','tile_wait_us','load_us_per_tile','walker_clk_per_step']})"
timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline --no-extra > gpurun_out/exp/cb2_c5.json 2> gpurun_out/exp/cb2_c5.err || { tail -20 gpurun_out/exp/cb2_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/exp/cb2_c5.json'));print('c5', round(d['ms_per_step'],3), 'walk', round(d['walk_ms'],3), d['config']['traceback_pin']['matches_oracle'])"
