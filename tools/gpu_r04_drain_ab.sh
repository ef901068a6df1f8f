#!/bin/bash
# Round 4: the drainer (bench_receiver drain, Sha1File through the digest queue) with the new default
# digest queue (1 GiB, 256 KiB chunks) against round 3's (256 MiB, 64 KiB), interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_drain_ab}
mkdir -p "$O"
D=/dev/shm/efes_drain_ab
rm -rf $D; mkdir -p $D
python3 - $D <<'PY'
import os, sys
d = sys.argv[1]
blob = os.urandom(4 << 20)  # every file the same bytes: the harness's sink answers with one digest
for i in range(256):
    open(os.path.join(d, f"{i}.fid"), "wb").write(blob)
PY
for rep in 1 2; do
  for q in "256 64" "1024 256"; do
    set -- $q
    for k in 16 128 512; do
      EFES_DIGEST_STAGING_MIB=$1 EFES_DIGEST_CHUNK_KIB=$2 timeout -k 10 200 tools/bench_receiver drain $D $k $((16 * k)) 4194304 256 \
        > "$O/q$2_k$k.$rep.json" 2> "$O/q$2_k$k.$rep.err" || { echo FAIL; tail -3 "$O/q$2_k$k.$rep.err"; rm -rf $D; exit 1; }
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d.get('value'), 'GiB/s', {k: d[k] for k in d if k in ('jobs_per_launch','cpu_s_per_gib','all_sums_equal','errors')})" "$O/q$2_k$k.$rep.json" "chunk_kib=$2 K=$k" | tee -a "$O/ab.log"
    done
  done
done
rm -rf $D
