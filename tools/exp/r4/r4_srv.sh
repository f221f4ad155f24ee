set -o pipefail
# round 4: recompute workers / window at 4-column stripes (C3 single call)
O=gpurun_out/r4_srv
mkdir -p $O
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-extra > $O/c3_$tag.json 2> $O/c3_$tag.err || { tail -5 $O/c3_$tag.err; return 1; }
  python3 -c "
import json
d=json.loads(open('$O/c3_$tag.json').read().strip().splitlines()[-1])
print('$tag', 'call', round(d['ms_per_step'],3), 'fill', round(d['fill_ms'],3), 'walk', round(d['walk_ms'],3), 'pin', d['config']['traceback_pin']['matches_oracle'])
"
}
run s64 GA_X=0 || exit 1
run s32 GA_RC_SERVERS=32 || exit 1
run s48 GA_RC_SERVERS=48 || exit 1
run s96 GA_RC_SERVERS=96 || exit 1
run s128 GA_RC_SERVERS=128 || exit 1
run w32 GA_RC_WIN=32 || exit 1
run e128 GA_RC_EVERY=128 || exit 1
run s64b GA_X=1 || exit 1
