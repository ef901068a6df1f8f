#!/bin/bash
# Round 6 robustness on the final library (the JIT dispatcher, the reclaim hand-over outside the
# registry lock): a long random fuzz of the fused digest pairs (3 000 scripts from 8 threads with the
# default 256 KiB staging chunks and 3 000 with 64 KiB chunks, seeds beyond the test suite's, every text
# and digest against the oracle).  ThreadSanitizer over the same library: tools/gpu_r06_jit_ab3.sh.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:?}" || exit 1
O=gpurun_out/${1:-r06_robust}
mkdir -p "$O"
for kib in 256 64; do
  EFES_DIGEST_CHUNK_KIB=$kib timeout -k 10 300 python3 -u - $kib > "$O/fuzz_$kib.log" 2>&1 <<'PY' || { tail -30 "$O/fuzz_$kib.log"; exit 1; }
import random, sys, threading, time
sys.path[:0] = [".", "tests"]
from oracle import oracle
oracle.build()
import efes_amd
from efes_amd import _lib, hashing
import test_gpu_pairs as T
kib = sys.argv[1]
base = {"256": 500_000, "64": 600_000}[kib]
gpu = dict(efes=efes_amd, hashing=hashing, lib=_lib.lib(), check=_lib.check, oracle_lib=oracle.lib())
s0 = hashing.pair_stats(); errors = []; t0 = time.time()
def worker(t):
    try:
        for k in range(t, 3000, 8):
            T._script(gpu, oracle, random.Random(base + k), 24, tag=f"{kib}K seed {base + k}")
    except Exception as e:
        errors.append(repr(e)[:2000])
ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
[th.start() for th in ths]; [th.join() for th in ths]
s1 = hashing.pair_stats()
print(f"{kib} KiB chunks", {k: s1[k] - s0[k] for k in s0}, "errors", len(errors), "seconds %.1f" % (time.time() - t0))
if errors: print(errors[:3]); sys.exit(1)
PY
  tail -1 "$O/fuzz_$kib.log"
done
echo fuzz done
