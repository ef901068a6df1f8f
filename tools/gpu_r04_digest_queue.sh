#!/bin/bash
# Round 4: the unchanged Go surface (tools/bench_go_surface, fused pairs) by digest-queue sizing
# (EFES_DIGEST_CHUNK_KIB / EFES_DIGEST_STAGING_MIB) and uploads in flight, 4 MiB single-PATCH uploads.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r04_digest_queue}
mkdir -p "$O"
for spec in "64 256" "128 512" "256 1024" "256 8208"; do
  set -- $spec
  for tk in "32 16" "32 64" "32 128" "32 256"; do
    set -- $spec $tk
    U=$(( $3 * $4 * 2 ))
    timeout -k 10 120 tools/bench_go_surface $3 $U 4194304 32768 $4 1 $1 $2 > "$O/q$1_$2_t$3_k$4.json" 2> "$O/q$1_$2_t$3_k$4.err" || { echo "FAIL $spec $tk"; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], 'in flight', sys.argv[3], d['value'], 'GiB/s', 'settles', d['settles'], 'hashed/byte', d['hashed_bytes_per_byte'], 'ok', d['all_equal'])" "$O/q$1_$2_t$3_k$4.json" "chunk_kib=$1 staging_mib=$2" $(( $3 * $4 )) | tee -a "$O/sweep.log"
  done
done
