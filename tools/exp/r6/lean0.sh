set -o pipefail
# round 6: the lean ramp (lean0: lean sub-chunks from the first step when row 0 is uniform) against the masked ramp,
# lane stamps of the C3 shape; the threaded tie-break table on the box's cores; the GPU suite; C3 / C5 / C2 lines
export TMPDIR=/tmp
O=gpurun_out/r6_lean0
mkdir -p $O
timeout -k 10 120 ./globalign_amd/_lib/ga_host_selftest bench 200001 > $O/rng_bench.txt 2>&1 || { cat $O/rng_bench.txt; exit 1; }
cat $O/rng_bench.txt
st() {
  name=$1; shift
  env GA_FILL_MODE=lane GA_LANE_COLS_PER_LANE=4 "$@" timeout -k 10 120 python -u tools/lane_stamps.py 100000 100000 > $O/stamps_$name.json 2> $O/stamps_$name.err || { tail -5 $O/stamps_$name.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/stamps_$name.json').read().strip().splitlines()[-1])
s=d['steady_state']
print('$name', 'plain', round(d['fill_ms_plain'],3), 'dbg', round(d['fill_ms_dbg'],3), 'first64', round(s.get('ns_per_step_first64_median',0),1), 'next64', round(s.get('ns_per_step_next64_median',0),1), 'end lags intra/cross', round(d['end_lag_intra_wg_us'],2), round(d['end_lag_cross_wg_us'],2), 'last end', round(d['last_end_us'],1))
for k,v in d['lag_by_row'].items(): print('   lag at row', k, {a: round(b,2) for a,b in v.items()})
"
}
st lean0
st ramp GA_OPTIONS="GA_LANE_LEAN0=0"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_suite.txt 2>&1 || { tail -40 $O/gpu_suite.txt; exit 1; }
tail -1 $O/gpu_suite.txt
for w in c3 c5 c2; do
  for v in 1 0; do
    timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-extra --opt GA_LANE_LEAN0=$v > $O/bench_${w}_$v.json 2> $O/bench_${w}_$v.err || { tail -20 $O/bench_${w}_$v.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('$O/bench_${w}_$v.json').read().strip().splitlines()[-1])
print('$w lean0=$v', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'tiebreak', round(d.get('host_tiebreak_ms',0),3), (d['config'].get('traceback_pin') or {}).get('matches_oracle'), d['config'].get('cost_matches_oracle'))
"
  done
done
