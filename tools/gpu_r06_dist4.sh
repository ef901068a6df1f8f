#!/bin/bash
# Round 6: the N>1 bench path rehearsed with 4 ranks on the one GPU (gloo for the timing barrier, the
# max-over-ranks and the per-rank record gather; the driver's 8-GPU run uses RCCL): every rank's record
# in the line, the rehearsal flag in ranks_check, exit 0.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r06_dist4}
mkdir -p "$O"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 4 --steps 5 --warmup 1 --dist-backend gloo --all-ranks-on-device0 --ingest-scale 0.05 \
  > "$O/dist4.json" 2> "$O/dist4.err" || { echo "dist4 failed"; tail -20 "$O/dist4.err"; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/dist4.json').read().strip().splitlines()[-1])
print('value', d['value'], 'n_gpus', d['n_gpus'], 'ingest', d['ingest_config']['value'])
for r in d['ranks']: print(r)
print(d['ranks_check'])"
