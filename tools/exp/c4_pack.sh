set -o pipefail
run() { tag=$1; shift; env "$@" timeout -k 10 120 python -u tools/fill_sweep.py 1000000 1000000 3 0 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['kind'], [round(x,2) for x in d['fill_ms']], d['cost'])" || exit 1; }
run default
run nwc4x2_sub8 GA_FILL_NWC=4 GA_LANE_WG_PER_CU=2 GA_FILL_LDS_FLOOR=0 GA_LANE_QROWS=2048 GA_LANE_SUB=8
run nwc4x2_sub16 GA_FILL_NWC=4 GA_LANE_WG_PER_CU=2 GA_FILL_LDS_FLOOR=0 GA_LANE_QROWS=2048
run td4_nwc8x2_sub16 GA_LANE_COLS_PER_LANE=4 GA_FILL_NWC=8 GA_LANE_WG_PER_CU=2 GA_FILL_LDS_FLOOR=0 GA_LANE_QROWS=1024
GA_FILL_NWC=4 GA_LANE_WG_PER_CU=2 GA_FILL_LDS_FLOOR=0 GA_LANE_QROWS=2048 GA_LANE_SUB=8 GA_FILL_MODE=lane timeout -k 10 120 python -u tools/lane_stamps.py 1000000 1000000 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:(round(v['cyc_per_step_busy'],1), round(v['wait_edge_frac'],3)) for k,v in d['by_simd'].items()}, d['by_wave'])"
