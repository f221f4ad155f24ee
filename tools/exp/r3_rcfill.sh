# STALE: the knobs this script sets were removed from ga_host.cpp in round 4, so it now measures the
# default path; kept only as the record of the measurement DESIGN.md cites.
# Round 3: what the recompute checkpoints cost the C3 fill (timing only: the walks of the DBG runs are wrong)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r3_rcfill.txt
: > $O
for cfg in "GA_RC=1" "GA_RC=1 GA_RC_DBG_NOCOL=1" "GA_RC=1 GA_RC_DBG_NOST=1" "GA_RC=1 GA_RC_DBG_NOCOL=1 GA_RC_DBG_NOST=1" "GA_RC=1 GA_LANE_COLS_PER_LANE=4"; do
  echo "== $cfg" >> $O
  env $cfg timeout -k 10 120 python -u tools/exp/r3_rc_diag.py 100000 96:48:1 >> $O 2>&1 || exit 1
done
