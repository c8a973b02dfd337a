#!/bin/bash
# round 6, call 37: the N>1 bench path end to end with this round's host changes (native driver,
# kernel staging, NUMA placement): 2 and 4 ranks sharing the one GPU (--same-device)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/n2_rehearsal.sh r06z12 > /dev/null && python -c "
import json; d=json.load(open('gpurun_out/n2_r06z12.json')); print('n2', d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d.get('driver'), d.get('main_thread'), d['config'].get('ba_exchange'))" || exit 1
bash tools/n4_rehearsal.sh r06z12 > /dev/null && python -c "
import json; d=json.load(open('gpurun_out/n4_r06z12.json')); print('n4', d['value'], d['value_reps_min'], d['value_reps_max'], d['ba_ms_per_iter'], d.get('driver'), d.get('main_thread'))" || exit 1
